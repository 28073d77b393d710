"""Headline benchmark: env-steps/sec, 2-player Splendor, 65536 tables per MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--tables T] [--players P] [--mode rollout|step] [--only]
    torchrun --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

One "step" = one SplendorEnv.step on every table of the batch (BASELINE.json config 3: legal
mask + uniform-random policy, same-step autoreset, obs int32[297] + mask int8[45] + reward +
terminated + flags written per table-step, terminal rows to final_obs).  Actions come from the
device policy (Philox over the new mask).  Two launch shapes compute the same trajectories and
write the same per-step outputs (tests/test_gpu_parity.py::test_rollout_equals_step_chain):
  --mode rollout  (headline) one spl_rollout launch per 16 env steps: state stays in registers
                  and each step's stores drain while the next step computes
  --mode step     one spl_step launch per env step (the drop-in SplendorEnv.step path);
                  the mode not selected is measured too and reported as "other_mode"
plus a pool refill every 64 steps (2p; 32 at 3p, 16 at 4p).  Inputs are resident in HBM before the timed region; the
timed region replays captured HIP graphs of 64 steps.

Weak scaling: each rank owns `--tables` tables (global ids rank*T ...), no collective in the
step path; after the timed region one all-gather (RCCL) collects episode returns.  value =
tables x world x steps / max-over-ranks wall time.

Printed on rank 0: ONE JSON line with the roofline of the mode's kernel (HIP events around each
launch of an eager window right after the timed replays; algorithmic bytes per SURVEY.md §8d:
1370 B per 2-player table-step) and, at N=1, the CPU baseline (the C oracle port, one process
per core).
"""
import argparse
import ctypes
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
for _p in (REPO, os.path.join(REPO, "splendor-gym_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level table)
ALGO_BYTES = {2: 1370, 3: 1408, 4: 1446}  # 2*S_P + 297*4 + 45 + 4 + 4 + 1 (3p interpolated)
# pool refill period per player count: three pool deals per table must cover the resets between
# refills (random games last ~77 plies at 2p, ~29 at 4p)
REFILL_EVERY = {2: 64, 3: 32, 4: 16}
ROLLOUT_K = 64     # env steps per spl_rollout launch (one fused pool refill per launch at 2p)


def cpu_baseline(players, procs, steps_per_proc):
    """The C oracle (a port of the reference engine) as `procs` single-env random rollouts,
    one process per core, started BEFORE this process touches the GPU (fork-safe)."""
    import multiprocessing as mp
    ctx = mp.get_context("fork")
    q = ctx.Queue()

    def work(i):
        import numpy as np
        from oracle.oracle import Oracle, pcg_state_of
        o = Oracle()
        pcg = np.array(pcg_state_of(1000 + i), np.uint64)
        eps = ctypes.c_int64()
        t = time.perf_counter()
        n = o.L.orc_random_rollout(players, pcg.ctypes.data, 7 + i, steps_per_proc, ctypes.byref(eps))
        q.put((n, time.perf_counter() - t, eps.value))

    ps = [ctx.Process(target=work, args=(i,)) for i in range(procs)]
    t0 = time.perf_counter()
    for p in ps:
        p.start()
    res = [q.get(timeout=600) for _ in ps]
    wall = time.perf_counter() - t0
    for p in ps:
        p.join()
    total = sum(r[0] for r in res)
    per_core = sum(r[0] / r[1] for r in res) / len(res)
    return {"value": round(total / wall, 1), "unit": "env-steps/s", "cores": procs, "kind": "port",
            "per_core": round(per_core, 1),
            "sample": (f"C oracle (port of engine/rules.py + envs/splendor_env.py step), {players}p, "
                       f"{procs} processes x {steps_per_proc} env steps, 1 env each, uniform-random legal "
                       f"policy with autoreset ({sum(r[2] for r in res)} episodes); reference Python "
                       "engine measured at 5.4k steps/s/core in SURVEY.md §6")}


def load_pmc_traffic(players, tables, mode, steps_per_launch):
    """HBM bytes per launch of the mode's kernel from the committed rocprofv3 PMC summary."""
    path = os.path.join(REPO, "profiles", "pmc_summary.json")
    kern = "k_step" if mode == "step" else "k_rollout"
    try:
        with open(path) as f:
            d = json.load(f)
        if (d.get("players") == players and d.get("tables") == tables
                and d.get("steps_per_launch", {}).get(kern) == steps_per_launch):
            return d.get("hbm_bytes_per_launch", {}).get(kern), os.path.relpath(path, REPO)
    except (OSError, ValueError, AttributeError):
        pass
    return None, None


def main():
    global ROLLOUT_K
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1024)
    ap.add_argument("--warmup", type=int, default=128)
    ap.add_argument("--tables", type=int, default=65536, help="tables per GPU")
    ap.add_argument("--players", type=int, default=2)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-procs", type=int, default=0, help="0 = min(16, cpu_count)")
    ap.add_argument("--cpu-steps", type=int, default=1_000_000, help="env steps per CPU process")
    ap.add_argument("--graph-steps", type=int, default=128,
                    help="steps per captured HIP graph (multiple of 128); 0 = eager launches")
    ap.add_argument("--mode", choices=("step", "rollout"), default="rollout",
                    help="rollout: one spl_rollout launch per "
                         f"{ROLLOUT_K} env steps; step: one spl_step launch per env step (same trajectories "
                         "and per-step outputs, tests/test_gpu_parity.py::test_rollout_equals_step_chain)")
    ap.add_argument("--only", action="store_true", help="skip measuring the other mode (reported as other_mode)")
    ap.add_argument("--rollout-k", type=int, default=ROLLOUT_K, help="env steps per spl_rollout launch")
    ap.add_argument("--refill-every", type=int, default=0, help="0 = per player count (64/32/16)")
    ap.add_argument("--refill", choices=("fused", "separate"), default="fused",
                    help="rollout mode: due pool refills run inside the spl_rollout launch (fused) or as a "
                         "spl_refill launch after it (step mode always launches spl_refill)")
    ap.add_argument("--pipeline", choices=("auto", "always", "half", "off"), default="auto",
                    help="rollout mode: two-wave pipelined kernel (auto: 32 or 64 tables per workgroup by grid "
                         "size; always: 64; half: 32) vs one wave per 64 tables (off)")
    args = ap.parse_args()
    ROLLOUT_K = args.rollout_k

    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    rank_env = int(os.environ.get("RANK", "0"))
    cpu = None
    if world_env == 1 and rank_env == 0 and not args.no_cpu_baseline:
        procs = args.cpu_procs or min(16, os.cpu_count() or 1)
        cpu = cpu_baseline(args.players, procs, args.cpu_steps)

    import torch
    from splendor_gym import _native
    from splendor_gym.device import Engine
    from splendor_gym.parallel import barrier, gather_returns, init_distributed, local_device, max_over_ranks

    rank, world, local = init_distributed()
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    dev = local_device(local)
    torch.cuda.set_device(dev)
    T, P = args.tables, args.players
    R = args.refill_every or REFILL_EVERY[P]
    table0 = rank * T
    # the library schedules the pool refills: every R steps (spl_step: a spl_refill launch; spl_rollout:
    # inside the rollout launch unless --refill separate)
    pipe = {"auto": True, "always": "always", "half": "half", "off": False}[args.pipeline]
    eng = Engine(T, P, device=dev, refill_period=R, table0=table0, refill_fused=args.refill == "fused",
                 pipeline=pipe)
    eng.reset(seeds=range(table0, table0 + T))
    lib = eng.lib
    buf = [torch.zeros(T, dtype=torch.int32, device=dev) for _ in range(2)]
    eng.sample_uniform(out=buf[0], seed=args.seed, ply=0)
    ep_ret = torch.zeros(T, dtype=torch.float32, device=dev)
    ep_cnt = torch.zeros(T, dtype=torch.int32, device=dev)
    ply_base = torch.zeros(1, dtype=torch.int64, device=dev)  # policy counter base, advanced per replay

    def mkargs(a_in, a_out):
        return _native.StepArgs(actions=a_in.data_ptr(), obs=eng.obs.data_ptr(), mask=eng.mask.data_ptr(),
                                reward=eng.reward.data_ptr(), terminated=eng.terminated.data_ptr(),
                                flags=eng.flags.data_ptr(), winner=eng.winner.data_ptr(),
                                final_obs=eng.final_obs.data_ptr(), autoreset=1, next_actions=a_out.data_ptr(),
                                ply_base=ply_base.data_ptr(), policy_seed=args.seed, ply=0, table0=table0,
                                ep_return=ep_ret.data_ptr(),
                                ep_count=ep_cnt.data_ptr())

    step_args = [mkargs(buf[0], buf[1]), mkargs(buf[1], buf[0])]
    ctx, desc = eng.ctx, ctypes.byref(eng.desc)
    stream = eng.stream()

    def run(mode, k0, k1, strm, ev=None):
        """Steps k0..k1-1 (ply k+1 relative to ply_base).  mode "step": one spl_step launch per
        step; "rollout": one spl_rollout launch per ROLLOUT_K steps.  Refills every R steps are
        issued by the library (the arena's step counter)."""
        per = 1 if mode == "step" else ROLLOUT_K
        for i, k in enumerate(range(k0, k1, per)):
            sa = step_args[(k // per) & 1]
            sa.ply = k + 1
            if ev is not None:
                ev[0][i].record()
            if mode == "step":
                _native.check(lib, lib.spl_step(ctx, desc, ctypes.byref(sa), strm))
            else:
                _native.check(lib, lib.spl_rollout(ctx, desc, ctypes.byref(sa), ROLLOUT_K, 0, strm))
            if ev is not None:
                ev[1][i].record()

    def measure(mode, k_base):
        """Warm up, capture, time K steps; returns the timing record.  Steps are numbered from
        k_base so every measurement continues the same trajectories (ply_base)."""
        W = (args.warmup // (2 * R)) * (2 * R)  # action-buffer parity and refill alignment
        ply_base.fill_(k_base)
        run(mode, 0, W, stream)
        K, G = args.steps, args.graph_steps
        graph, how = None, "eager"
        if G > 0:
            if G % (2 * R) or K % G:
                raise SystemExit(f"--graph-steps must be a multiple of {2 * R} that divides --steps")
            try:
                torch.cuda.synchronize(dev)
                ply_base.fill_(k_base + W)
                graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(graph):
                    run(mode, 0, G, ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream))
                    ply_base.add_(G)
                how = f"hipGraph replays of {G} steps"
            except Exception as exc:  # capture unsupported: time eager launches instead
                print(f"graph capture failed ({exc}); timing eager launches", file=sys.stderr)
                graph, G = None, 0
        per = 1 if mode == "step" else ROLLOUT_K
        barrier(dev)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        if graph is not None:
            for _ in range(K // G):
                graph.replay()
            ev = None
        else:
            ev = ([torch.cuda.Event(enable_timing=True) for _ in range(K // per)],
                  [torch.cuda.Event(enable_timing=True) for _ in range(K // per)])
            ply_base.fill_(k_base + W)
            run(mode, 0, K, stream, ev)
        torch.cuda.synchronize(dev)
        barrier(dev)
        elapsed = max_over_ranks(time.perf_counter() - t0, device=dev)
        if ev is None:
            # ROCm rejects timing events as graph nodes ("External events are disallowed"), so the
            # kernel duration comes from HIP events around each launch of an eager window of the
            # same loop, run right after the timed replays on the same stream and state.
            nwin = max(64, 4 * per)  # at least four launches
            ev = ([torch.cuda.Event(enable_timing=True) for _ in range(nwin // per)],
                  [torch.cuda.Event(enable_timing=True) for _ in range(nwin // per)])
            ply_base.fill_(k_base + W + K + 1)
            run(mode, 0, nwin, stream, ev)
            torch.cuda.synchronize(dev)
        nev = len(ev[0])
        launch_s = sum(ev[0][i].elapsed_time(ev[1][i]) for i in range(nev)) / nev / 1e3
        return {"mode": mode, "elapsed": elapsed, "launch_s": launch_s, "steps_per_launch": per, "how": how,
                "nev": nev, "k_next": k_base + W + K + 1 + max(64, 4 * per) + 1}

    main_rec = measure(args.mode, 0)
    alt_rec = None
    if not args.only:
        alt_rec = measure("rollout" if args.mode == "step" else "step", main_rec["k_next"])
    K = args.steps
    # correctness canaries on the measured run: no error flags, episodes completed
    bad = int(((eng.flags & (_native.F_OOB | _native.F_AFTER_TERMINAL | _native.F_RNG_LIMIT)) != 0).sum().item())
    rets, cnts = gather_returns(ep_ret, ep_cnt.to(torch.int64), n_global=T * world)
    episodes = int(cnts.sum().item())

    def summary(rec):
        total_steps = T * world * K
        algo = ALGO_BYTES[P] * T * rec["steps_per_launch"]
        rk = "k_rollout" if args.pipeline == "off" else "k_rollout_ws"  # two-wave pipelined kernel
        kname = f"spl::k_step<{P}>" if rec["mode"] == "step" else f"spl::{rk}<{P}> ({ROLLOUT_K} steps per launch)"
        return {"mode": rec["mode"], "value": round(total_steps / rec["elapsed"], 1),
                "ms_per_step": round(rec["elapsed"] / K * 1e3, 4),
                "roofline": {"bound": "hbm", "achieved": round(algo / rec["launch_s"] / 1e9, 1),
                             "peak": HBM_PEAK_GBS, "unit": "GB/s",
                             "frac": round(algo / rec["launch_s"] / 1e9 / HBM_PEAK_GBS, 4),
                             "kernel": kname, "kernel_avg_us": round(rec["launch_s"] * 1e6, 2),
                             "kernel_timing": ("HIP events around each launch in the timed region" if rec["how"] == "eager"
                                               else f"HIP events around each of {rec['nev']} eager launches right "
                                                    "after the timed replays"),
                             "algo_bytes_per_launch": algo},
                "launch": rec["how"]}

    if rank == 0:
        main = summary(main_rec)
        traffic, traffic_src = load_pmc_traffic(P, T, main_rec["mode"], main_rec["steps_per_launch"])
        roof = dict(main["roofline"], traffic=traffic, traffic_source=traffic_src)
        out = {
            "metric": f"env-steps/sec (whole node), {P}p {T} tables/GPU",
            "value": main["value"],
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": K,
            "warmup": args.warmup,
            "ms_per_step": main["ms_per_step"],
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic: seeded deals (table id = env seed), device uniform-random legal policy",
            "config": {"workload": f"{P}-player SplendorEnv.step x {T} tables per GPU, legal mask + uniform-random "
                                   "policy, same-step autoreset, obs int32[297] + mask int8[45] per table-step",
                       "tables_per_gpu": T, "players": P, "parallelism": f"table-sharded x{world}",
                       "refill_every": R, "refill": args.refill if main_rec["mode"] == "rollout" else "separate", "pipeline": args.pipeline,
                       "rollout_steps_per_launch": ROLLOUT_K, "mode": main["mode"],
                       "launch": main["launch"]},
            "roofline": roof,
            "cpu_baseline": cpu,
            "episodes": episodes,
            "mean_final_reward_p0": round(float(rets.sum().item()) / max(1, episodes), 4),
            "error_flags": bad,
        }
        if alt_rec is not None:
            out["other_mode"] = summary(alt_rec)
        print(json.dumps(out))
    eng.close()
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
