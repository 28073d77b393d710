"""Time the fused ActorCritic kernel (spl_policy_act) against the torch module on engine
observations:  python tools/bench_policy.py [--tables 65536] [--iters 50]

Prints one JSON line: per-call microseconds and achieved TFLOP/s (algorithmic: 2 x MACs of the
unpadded 297-256-256-45 actor (+ 297-256-256-1 critic) per table) for SAMPLE (actor + critic) and
GREEDY (actor), next to torch fp32 and bf16-autocast get_action_and_value / greedy."""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "splendor-gym_amd")]

MACS_ACTOR = 297 * 256 + 256 * 256 + 256 * 45
MACS_CRITIC = 297 * 256 + 256 * 256 + 256


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tables", type=int, default=65536)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--fused-only", action="store_true", help="skip the torch timings")
    ap.add_argument("--config5-only", action="store_true",
                    help="only config 5's agent call: trained weights, compact rows, sample + critic (for PMC passes)")
    args = ap.parse_args()
    import torch
    from splendor_gym.device import Engine
    from splendor_gym.fused_policy import FusedActorCritic
    from splendor_gym.policy import ActorCritic, greedy_actions

    n = args.tables
    e = Engine(n, 2)
    e.reset(seeds=range(n))
    a = torch.zeros(n, dtype=torch.int32, device=e.device)
    e.sample_uniform(out=a, seed=1, ply=0)
    for k in range(8):
        e.step(a, next_actions=a, policy_seed=1, ply=k + 1)
    obs, mask = e.obs, e.mask
    torch.manual_seed(0)
    m = ActorCritic().to(e.device).eval()
    f = FusedActorCritic(m)                             # fp32: exact operands, three bf16 planes
    fh = FusedActorCritic(m, precision="fp32_f16x2")    # fp32 within 2^-22: two fp16 planes
    f16 = FusedActorCritic(m, precision="bf16")         # opt-in bf16 MFMA

    def timeit(fn):
        for _ in range(5):
            fn()
        s, t = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s.record()
        for _ in range(args.iters):
            fn()
        t.record()
        torch.cuda.synchronize()
        return s.elapsed_time(t) * 1e3 / args.iters

    res = {}
    if args.config5_only:
        from safetensors.torch import load_file
        u8 = torch.zeros(n, 300, dtype=torch.uint8, device=e.device)
        e.step(a, next_actions=a, policy_seed=1, ply=9, obs_u8=u8)
        mt = ActorCritic().to(e.device).eval()
        mt.load_state_dict(load_file(os.path.join(REPO, "tests", "golden", "ppo_splendor_latest.safetensors"),
                                     device=str(e.device)))
        ft = FusedActorCritic(mt)
        res["trained_fp32_sample_u8obs_us"] = timeit(lambda: ft.act(u8, mask, seed=1, ply=2))
        print(json.dumps(res))
        return 0
    res["fused_fp32_sample_us"] = timeit(lambda: f.act(obs, mask, seed=1, ply=2))
    res["fused_fp32_greedy_us"] = timeit(lambda: f.greedy(obs, mask))
    res["fused_fp32_f16x2_sample_us"] = timeit(lambda: fh.act(obs, mask, seed=1, ply=2))
    res["fused_fp32_f16x2_greedy_us"] = timeit(lambda: fh.greedy(obs, mask))
    res["fused_bf16_sample_us"] = timeit(lambda: f16.act(obs, mask, seed=1, ply=2))
    res["fused_bf16_greedy_us"] = timeit(lambda: f16.greedy(obs, mask))
    # the same calls on compact uint8 observation rows (Engine.step obs_u8: 300 B per table instead of
    # 1 188; one more step writes them, so they are the next state's, timed alike)
    u8 = torch.zeros(n, 300, dtype=torch.uint8, device=e.device)
    e.step(a, next_actions=a, policy_seed=1, ply=9, obs_u8=u8)
    res["fused_fp32_sample_u8obs_us"] = timeit(lambda: f.act(u8, mask, seed=1, ply=2))
    res["fused_fp32_greedy_u8obs_us"] = timeit(lambda: f.greedy(u8, mask))
    res["fused_fp32_f16x2_sample_u8obs_us"] = timeit(lambda: fh.act(u8, mask, seed=1, ply=2))
    # the same state as int32 rows (bytes 0-296 widened, move_count's high byte at 297 folded in)
    o32 = u8[:, :297].to(torch.int32).contiguous()
    o32[:, 295] += 256 * u8[:, 297].to(torch.int32)
    res["fused_fp32_sample_samestate_int32_us"] = timeit(lambda: f.act(o32, mask, seed=1, ply=2))
    res["fused_fp32_greedy_samestate_int32_us"] = timeit(lambda: f.greedy(o32, mask))
    res["int32_obs_max"] = int(obs.max().item())
    res["int32_obs_min"] = int(obs.min().item())
    # the reference's trained weights (config 5's agent) on the same two forms of the same state
    from safetensors.torch import load_file
    mt = ActorCritic().to(e.device).eval()
    mt.load_state_dict(load_file(os.path.join(REPO, "tests", "golden", "ppo_splendor_latest.safetensors"),
                                 device=str(e.device)))
    ft = FusedActorCritic(mt)
    res["trained_fp32_sample_int32_us"] = timeit(lambda: ft.act(o32, mask, seed=1, ply=2))
    res["trained_fp32_sample_u8obs_us"] = timeit(lambda: ft.act(u8, mask, seed=1, ply=2))
    # the same call after 64 MB of other writes (the L2s hold none of the image: as in the dual step,
    # where the opponents' images pass through first), timed per launch with events around the call
    junk = torch.empty(64 << 20, dtype=torch.uint8, device=e.device)

    def timed_after_flush(fn, flush):
        ts = []
        for i in range(args.iters + 5):
            if flush:
                junk.fill_(i & 255)
            s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s0.record()
            fn()
            s1.record()
            torch.cuda.synchronize()
            if i >= 5:
                ts.append(s0.elapsed_time(s1) * 1e3)
        return sorted(ts)[len(ts) // 2]
    res["trained_fp32_sample_u8obs_warm_median_us"] = timed_after_flush(lambda: ft.act(u8, mask, seed=1, ply=2), False)
    res["trained_fp32_sample_u8obs_flushed_median_us"] = timed_after_flush(lambda: ft.act(u8, mask, seed=1, ply=2), True)

    def torch_sample():
        with torch.no_grad():
            return m.get_action_and_value(obs.float(), mask.float())

    def torch_sample_bf16():
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
            return m.get_action_and_value(obs.float(), mask.float())

    if not args.fused_only:
        res["torch_fp32_sample_us"] = timeit(torch_sample)
        res["torch_bf16_sample_us"] = timeit(torch_sample_bf16)
        res["torch_fp32_greedy_us"] = timeit(lambda: greedy_actions(m, obs, mask))
    fl_s = 2.0 * n * (MACS_ACTOR + MACS_CRITIC)
    fl_g = 2.0 * n * MACS_ACTOR
    for p in ("fp32", "fp32_f16x2", "bf16"):
        res[f"fused_{p}_sample_tflops"] = fl_s / res[f"fused_{p}_sample_us"] / 1e6
        res[f"fused_{p}_greedy_tflops"] = fl_g / res[f"fused_{p}_greedy_us"] / 1e6
    res["peak_tflops"] = {"fp32": 157.3, "bf16": 2500.0}  # dense MFMA peaks (MI355X_MICROARCH.md)
    res["tables"] = n
    print(json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in res.items()}))


if __name__ == "__main__":
    main()
