"""The reference's trained ActorCritic weights (runs/ppo_splendor/ppo_splendor_latest.pt, the one
297-input checkpoint) as a data fixture for the GPU box, where the
reference does not exist.  Loaded with torch.load(weights_only=True) — nothing in the file is
executed — and re-saved as safetensors (12 fp32 tensors, actor.* and critic.*, state_dict names
of ppo_splendor.py:40-59).

    python tests/golden/make_golden_checkpoint.py        # here, with /root/reference

Writes tests/golden/ppo_splendor_latest.safetensors.
"""
import os

import torch
from safetensors.torch import save_file

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = "/root/reference/runs/ppo_splendor/ppo_splendor_latest.pt"


def main():
    sd = torch.load(SRC, map_location="cpu", weights_only=True)
    out = {k: v.detach().to(torch.float32).contiguous() for k, v in sd.items()}
    assert out["actor.0.weight"].shape == (256, 297) and out["critic.4.weight"].shape == (1, 256)
    save_file(out, os.path.join(HERE, "ppo_splendor_latest.safetensors"), metadata={"source": SRC})
    print({k: tuple(v.shape) for k, v in out.items()})


if __name__ == "__main__":
    main()
