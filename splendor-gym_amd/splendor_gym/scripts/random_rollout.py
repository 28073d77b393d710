"""Uniform-random episodes on the GPU-backed SplendorEnv (reference scripts/random_rollout.py:7-30):
episode ep resets with seed + ep, plays numpy-uniform legal moves for at most 500 plies, and prints
the steps and last reward.  BASELINE config 1 plumbing; the batched form is Engine.rollout."""
import argparse

import numpy as np

from ..envs import SplendorEnv


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--episodes", type=int, default=3)
    ap.add_argument("--seed", type=int, default=0)
    args = ap.parse_args(argv)
    env = SplendorEnv(num_players=2)
    wins = 0
    for ep in range(args.episodes):
        obs, info = env.reset(seed=args.seed + ep)
        steps, reward, done = 0, 0.0, False
        while not done and steps < 500:
            legal = np.flatnonzero(info["action_mask"])
            if len(legal) == 0:
                break
            obs, reward, terminated, truncated, info = env.step(int(np.random.choice(legal)))
            steps += 1
            done = terminated or truncated
        print(f"Episode {ep}: steps={steps} reward={reward}")
        wins += reward > 0
    print(f"Wins: {wins}/{args.episodes}")


if __name__ == "__main__":
    main()
