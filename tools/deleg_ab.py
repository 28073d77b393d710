"""Rollout-store delegation A/B on one box, arms alternating (VERDICT r02 "Next round" 2).

    python tools/deleg_ab.py [--rounds 12] [--arms 0,6] [--tables 65536]

One engine and one [128, T, ...] rollout store; each round runs one 128-step spl_rollout launch per
arm (order alternating between rounds), each bracketed by HIP events on the launch stream.  Prints
per-arm mean / sd / min of the launch time in µs and one JSON line.
"""
import argparse
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "splendor-gym_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=12)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--arms", default="0,6")
    ap.add_argument("--tables", type=int, default=65536)
    ap.add_argument("--players", type=int, default=2)
    a = ap.parse_args()
    import torch
    from splendor_gym import _native
    from splendor_gym.device import Engine
    T, P, K = a.tables, a.players, 128
    arms = [int(x) for x in a.arms.split(",")]
    eng = Engine(T, P, device="cuda:0", refill_period={2: 64, 3: 32, 4: 16}[P])
    eng.reset(seeds=range(T))
    dev = eng.device
    acts = [torch.zeros(T, dtype=torch.int32, device=dev) for _ in range(2)]
    eng.sample_uniform(out=acts[0], seed=3, ply=0)
    out = dict(obs=torch.empty((K, T, 297), dtype=torch.int32, device=dev),
               mask=torch.empty((K, T, 45), dtype=torch.int8, device=dev),
               reward=torch.empty((K, T), dtype=torch.float32, device=dev),
               terminated=torch.empty((K, T), dtype=torch.uint8, device=dev),
               flags=torch.empty((K, T), dtype=torch.uint8, device=dev),
               winner=torch.empty((K, T), dtype=torch.int8, device=dev),
               final_obs=torch.empty((K, T, 297), dtype=torch.int32, device=dev))
    times = {arm: [] for arm in arms}
    ply, i = 1, 0
    for r in range(a.warmup + a.rounds):
        order = arms if r % 2 == 0 else arms[::-1]
        for arm in order:
            _native.check(eng.lib, eng.lib.spl_ctx_set_rollout_delegation(eng.ctx, arm))
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            eng.rollout(K, actions=acts[i & 1], next_actions=acts[(i + 1) & 1], policy_seed=3, ply=ply, out=out)
            e1.record()
            torch.cuda.synchronize(dev)
            if r >= a.warmup:
                times[arm].append(e0.elapsed_time(e1) * 1e3)
            ply += K
            i += 1
        print(f"round {r}: " + ", ".join(f"{arm}: {times[arm][-1]:.1f}" for arm in arms if times[arm]),
              file=sys.stderr, flush=True)
    res = {}
    for arm in arms:
        v = times[arm]
        res[str(arm)] = {"n": len(v), "mean_us": round(statistics.mean(v), 1), "sd_us": round(statistics.stdev(v), 1),
                         "min_us": round(min(v), 1), "max_us": round(max(v), 1)}
        print(f"delegation {arm}: mean {res[str(arm)]['mean_us']} sd {res[str(arm)]['sd_us']} "
              f"min {res[str(arm)]['min_us']} (n={len(v)})")
    base = res[str(arms[0])]["mean_us"]
    for arm in arms[1:]:
        res[str(arm)]["gain_vs_first_arm"] = round(1 - res[str(arm)]["mean_us"] / base, 4)
    print(json.dumps({"tables": T, "players": P, "steps_per_launch": K, "arms": res,
                      "kernel": eng.rollout_kernel_name(True)}))
    eng.close()


if __name__ == "__main__":
    main()
