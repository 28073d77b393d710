"""The RCCL (backend "nccl") side of splendor_gym.parallel on the real device.

The bench's N > 1 path gathers device identities, episode returns and the slowest rank's time over
RCCL. The one-GPU box cannot start two RCCL ranks (RCCL refuses two ranks on one card), so this test
runs ONE rank of an RCCL group and makes the helpers take their collective branch anyway
(`parallel._single` patched): the same calls, device tensors and argument shapes that N ranks issue,
with a world of one. The gloo tests in test_host_cpu.py cover two real ranks on the CPU."""
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)

CHILD = r'''
import os, sys
sys.path[:0] = [sys.argv[1], os.path.join(sys.argv[1], "splendor-gym_amd")]
import torch
import torch.distributed as dist
from splendor_gym import parallel
os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=sys.argv[2])
torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
dist.init_process_group(backend="nccl", rank=0, world_size=1, device_id=dev)
assert dist.get_backend() == "nccl"
parallel._single = lambda: False  # take the N-rank branches with a world of one
census = parallel.device_census(parallel.device_identity(dev))
assert census["ranks"] == 1 and census["devices"] == 1 and not census["shared_device"], census
ret = torch.arange(1001, dtype=torch.float32, device=dev) * 0.5
cnt = torch.arange(1001, dtype=torch.int32, device=dev) % 7
r, c = parallel.gather_returns(ret, cnt, n_global=1001)
assert r.device == dev and torch.equal(r, ret) and torch.equal(c, cnt.to(torch.int64))
assert parallel.max_over_ranks(1.25, device=dev) == 1.25
parallel.barrier(dev)
torch.cuda.synchronize()
dist.destroy_process_group()
print("rccl ok", census["identities"][0])
'''


@pytest.mark.gpu
def test_rccl_collective_branches_on_one_rank():
    port = str(29900 + os.getpid() % 90)
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    r = subprocess.run([sys.executable, "-c", CHILD, REPO, port], env=env, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "rccl ok" in r.stdout
