"""Per-step time of the drop-in batched surface, SplendorVectorEnv.step (vector.py), against the bare
spl_step kernel: python tools/bench_vec_step.py [--tables 65536] [--steps 256]

Actions come from the device uniform policy (vec.sample_actions), so the loop is the env surface
alone: the step launch, the per-step error check of the reference's exceptions and the info dict."""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "splendor-gym_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tables", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=256)
    args = ap.parse_args()
    import torch
    from splendor_gym import SplendorVectorEnv
    out = {"tables": args.tables}
    for mode, copy in (("sync", True), ("deferred", True), ("sync", False), ("deferred", False)):
        vec = SplendorVectorEnv(args.tables, device="cuda:0", check_actions=mode, copy=copy)
        obs, info = vec.reset(seed=0)
        for k in range(32):  # warm-up
            obs, rew, term, trunc, info = vec.step(vec.sample_actions(seed=1, ply=k))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(args.steps):
            obs, rew, term, trunc, info = vec.step(vec.sample_actions(seed=1, ply=100 + k))
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / args.steps
        out[f"{mode}{'' if copy else '_nocopy'}"] = {"vector_env_step_us": round(dt * 1e6, 2),
                                                     "env_steps_per_s": round(args.tables / dt, 1)}
        vec.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
