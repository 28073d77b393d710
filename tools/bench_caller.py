"""bench.py's caller_path line alone (the unchanged ppo_splendor.py loop shape over SplendorEnv):
    python tools/bench_caller.py [--envs 16] [--iters 150] [--reps 3]"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "splendor-gym_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=16)
    ap.add_argument("--iters", type=int, default=150)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import bench
    for r in range(a.reps):
        line = bench.caller_path_line(n_envs=a.envs, iters=a.iters)
        print(json.dumps({k: line[k] for k in ("value", "us_per_splendorenv_step", "us_per_dual_step", "host_share")}
                         | {"rep": r}), flush=True)


if __name__ == "__main__":
    main()
