"""Where one SplendorEnv.step's time goes on the host (the unchanged ppo_splendor.py caller path):
launch (ctypes spl_step), wait (stream synchronize), and the rest (action write, output copies, info
dict), per call, medians over N calls with random legal actions.
    python tools/prof_env_step.py [N] [SHAPE]   (SHAPE: spl_ctx_set_step_tail mode, -1 = auto)"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "splendor-gym_amd")]


def main():
    import numpy as np
    import torch
    from splendor_gym.envs import SplendorEnv
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
    shape = int(sys.argv[2]) if len(sys.argv) > 2 else -1  # spl_ctx_set_step_tail mode (-1 auto)
    env = SplendorEnv()
    obs, info = env.reset(seed=0)
    rng = np.random.default_rng(0)
    e = env._eng
    e.lib.spl_ctx_set_step_tail(e.ctx, shape)
    launch0 = env._launch
    dev = e.device
    stamps = {"launch": [], "wait": []}

    def timed_launch():
        t0 = time.perf_counter_ns()
        launch0()
        t1 = time.perf_counter_ns()
        torch.cuda.current_stream(dev).synchronize()
        t2 = time.perf_counter_ns()
        stamps["launch"].append(t1 - t0)
        stamps["wait"].append(t2 - t1)
    total = []
    for phase in ("plain", "split"):
        env._launch = launch0 if phase == "plain" else timed_launch
        for k in range(n):
            legal = np.flatnonzero(info["action_mask"])
            if legal.size == 0:  # a drawn game (no legal move) ends at the next step; start a new one
                obs, info = env.reset()
                legal = np.flatnonzero(info["action_mask"])
            a = int(rng.choice(legal))
            t0 = time.perf_counter_ns()
            obs, r, term, trunc, info = env.step(a)
            t1 = time.perf_counter_ns()
            if phase == "plain":
                total.append(t1 - t0)
            if term:
                obs, info = env.reset()
    med = lambda v: float(np.median(v)) / 1e3
    print(json.dumps({"calls": n, "step_tail": shape, "step_us_median": med(total), "step_us_mean": float(np.mean(total)) / 1e3,
                      "launch_us_median": med(stamps["launch"]), "wait_us_median": med(stamps["wait"]),
                      "note": "launch = ctypes spl_step incl. hipLaunchKernel; wait = stream synchronize after it"}))


if __name__ == "__main__":
    main()
