"""Headline benchmark: env-steps/sec, 2-player Splendor, 65536 tables per MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--tables T] [--players P] [--mode rollout|step] [--only]
    torchrun --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

`--gpus N` with N > 1 and no launcher in the environment (no WORLD_SIZE) starts its own N ranks
(self_launch: one child process per GPU, this process never touches a GPU) and exits non-zero when
the node shows fewer than N GPUs or the ranks do not land on N distinct devices, instead of
reporting a one-GPU figure for an N-GPU request.  Under torchrun the ranks are the launcher's.

One "step" = one SplendorEnv.step on every table of the batch (BASELINE.json config 3: legal
mask + uniform-random policy, same-step autoreset, obs int32[297] + mask int8[45] + reward +
terminated + flags + winner written per table-step, terminal rows to final_obs).  Actions come
from the device policy (Philox over the new mask).  Two launch shapes compute the same
trajectories and write the same per-step outputs (tests/test_gpu_parity.py::test_rollout_equals_step_chain):
  --mode rollout  (headline) one spl_rollout launch per 128 env steps (one PPO rollout of
                  ppo_splendor.py's --num-steps 128): state stays in registers, each step's stores
                  drain while the next step computes, and step k's outputs go to block k of a
                  [128, T, ...] rollout store (≈20 GB at 65536 tables: far larger than the 256 MiB
                  Infinity Cache, so every output byte reaches HBM)
  --mode step     one spl_step launch per env step (the drop-in SplendorEnv.step path), timed as
                  captured HIP graphs of whole refill periods
The mode not selected is measured too ("other_mode"), and the rollout kernel is measured a second
time writing every step into the same [T, ...] block ("in_place_l3": that ~81 MB block stays
resident in the Infinity Cache, so it is NOT an HBM figure and is never the headline).  Two more
secondary lines: "config5_selfplay" (BASELINE config 5 per GPU: fused fp32 ActorCritic + batched
dual step with the opponent pool, hipGraph replays) and "config4_share" (BASELINE config 4's
per-GPU share: 4 players x 32768 tables, the same per-step rollout store, 8 launches timed).

--steps / --warmup are rounded UP to whole plan units (step_plan): a unit is two launches (the
action buffers alternate) and whole pool-refill periods; "steps" in the JSON line is the number
of env steps actually timed.  Warm-up is at least one unit (one full launch and one refill cycle).

Weak scaling: each rank owns `--tables` tables (global ids rank*T ...), no collective in the
step path; after the timed region one all-gather (RCCL) collects episode returns.  value =
tables x world x steps / max-over-ranks wall time.

Printed on rank 0: ONE JSON line with the roofline of the headline kernel (HIP events around each
launch inside the timed region, on the launch stream) and, at N=1, the CPU baseline (the C oracle
port, one process per core, bounded sample).
"""
import argparse
import ctypes
import json
import math
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
for _p in (REPO, os.path.join(REPO, "splendor-gym_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level table)
HBM_ACHIEVABLE_GBS = 6290.0    # the guide's measured float4-copy ceiling (MI355X_MICROARCH.md:36)
# canonical packed mutable state per table (S_2 = 64 B, S_4 = 102 B; 3p interpolated)
STATE_BYTES = {2: 64, 3: 83, 4: 102}
# per table-step outputs of both kernels: obs int32[297] + mask int8[45] + reward f32 + terminated u8
# + flags u8 + winner i8
OUT_BYTES = 297 * 4 + 45 + 4 + 1 + 1 + 1
OBS_ROW = 297 * 4
# SURVEY.md §8d drop-in figure for k_step: 2*S_P + obs + mask + action + reward + terminated, + 16 B of
# the legal-mask cache (round 6, ABI 9: 8 B read with the state, 8 B written with it; not part of S_P)
LEGAL_CACHE_BYTES = 16
STEP_ALGO_BYTES = {p: 2 * s + LEGAL_CACHE_BYTES + 297 * 4 + 45 + 4 + 4 + 1 for p, s in STATE_BYTES.items()}  # 2p: 1386
# pool refill period per player count: three pool deals per table must cover the resets between
# refills (random games last ~77 plies at 2p, ~29 at 4p)
REFILL_EVERY = {2: 64, 3: 32, 4: 16}
F16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X dense fp16/bf16 MFMA (MI355X_MICROARCH.md chip table; no sparsity)
# 16-bit MFMA work of the fused fp32 ActorCritic (csrc/spl_policy32.hip) per table, per operand format
# (precision): "fp32" = EXACT fp32 operands as three bf16 planes: layer 1 (297 -> 256, the observation
# exact in one plane) takes 3 plane products, layers 2 (256 -> 256) and 3 (256 -> 45) take the 6 of
# order <= 2; "fp32_f16x2" = two fp16 planes (22 significant bits): 2 and 3 products.  The critic's
# 256 -> 1 output runs on VALU, not counted.
MFMA_PRODUCTS = {"fp32": (3, 6), "fp32_f16x2": (2, 3)}


def actor_critic_mfma_flop(precision):
    """(actor, critic) 16-bit MFMA flop per table of get_action_and_value at `precision`."""
    l1, hid = MFMA_PRODUCTS[precision]
    return (2 * (297 * 256 * l1 + 256 * 256 * hid + 256 * 45 * hid), 2 * (297 * 256 * l1 + 256 * 256 * hid))


PRECISION_DTYPE = {
    "fp32": "fp32 (EXACT fp32 operands: three bf16 planes of 24 significant bits, the six plane products of "
            "order <= 2 accumulated in fp32, dropped terms <= 2^-24 of each product; tanh to a few ulp)",
    "fp32_f16x2": "fp32 within 2^-22 (two fp16 planes of 22 significant bits per operand, three plane products "
                  "accumulated in fp32; NOT an exact fp32 operand representation)"}
# the network's own fp32 work per table (2 x MACs of actor + critic), for the fp32-equivalent rate
NET_FP32_FLOP = 2 * (297 * 256 + 256 * 256 + 256 * 45 + 297 * 256 + 256 * 256 + 256)
ROLLOUT_K = 128    # env steps per spl_rollout launch = ppo_splendor.py's --num-steps default (:71)
MIN_TIMED_LAUNCHES = 8  # rollout mode times at least this many launches (>= 16 ms), whatever --steps says
MIN_TIMED_REPLAYS = 4   # step mode (hipGraphs) times at least this many replays of a full graph (~12 ms)


def step_plan(mode, steps, warmup, refill_period, rollout_k=ROLLOUT_K, graph_steps=128,
              min_launches=MIN_TIMED_LAUNCHES, min_replays=MIN_TIMED_REPLAYS):
    """Turn the requested --steps/--warmup into what is actually run.

    unit   = lcm(2 launches, refill period): the two action buffers alternate per launch, and a
             captured graph must hold whole refill periods (the library schedules refills from
             the arena's step counter, which the graph bakes in).
    K      = steps timed    = --steps rounded up to whole units (>= 1 unit), and to at least
             `min_launches` launches in rollout mode (the driver's --steps 20 would otherwise time
             two ~2 ms launches, where one box's jitter moves the figure by several percent) and to
             at least `min_replays` full graphs in step mode (one ~1.5 ms replay let a single stall
             move the figure by half)
    W      = warm-up steps  = --warmup rounded up to whole units (>= 1 unit: one full launch + a
             refill cycle, whatever --warmup says)
    G      = steps per captured graph (step mode only; 0 = eager launches): the largest multiple
             of unit that divides K and is <= max(graph_steps, unit); rollout mode is timed eagerly
             (one ~2 ms launch per 128 steps: launch overhead is hidden by the queue)
    launches = K / per (per = steps per launch)
    """
    if mode not in ("step", "rollout"):
        raise ValueError(mode)
    per = 1 if mode == "step" else int(rollout_k)
    if per <= 0:
        raise ValueError("rollout_k must be positive")
    r = int(refill_period)
    unit = 2 * per if r <= 0 else (2 * per) * r // math.gcd(2 * per, r)
    k = max(1, -(-max(int(steps), 1) // unit)) * unit
    if mode == "rollout":
        k = max(k, -(-int(min_launches) * per // unit) * unit)
    w = max(1, -(-max(int(warmup), 0) // unit)) * unit
    g = 0
    if mode == "step" and graph_steps and graph_steps > 0:
        cap = max(int(graph_steps), unit)
        k = max(k, int(min_replays) * (cap // unit) * unit)
        g = unit
        m = unit
        while m <= min(cap, k):
            if k % m == 0:
                g = m
            m += unit
    return {"mode": mode, "per": per, "unit": unit, "K": k, "W": w, "G": g, "launches": k // per,
            "requested_steps": int(steps), "requested_warmup": int(warmup)}


def _cpu_leg(players, procs, steps_per_proc):
    """`procs` single-env random rollouts of the C oracle, one process each (fork, before any GPU
    use); returns (env steps, wall seconds, mean per-process rate, episodes)."""
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
    return (sum(r[0] for r in res), wall, sum(r[0] / r[1] for r in res) / len(res), sum(r[2] for r in res))


def cgroup_cpu_quota():
    """CPUs the cgroup CPU quota grants this process (cgroup v2 /sys/fs/cgroup/cpu.max "quota period",
    or v1 cpu.cfs_quota_us / cpu.cfs_period_us), with the file it came from; (None, source) when the
    quota is unlimited or not readable."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        return (None if q == "max" else int(q) / int(per)), "/sys/fs/cgroup/cpu.max: " + q + " " + per
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            per = int(f.read())
        return (None if q <= 0 else q / per), f"/sys/fs/cgroup/cpu/cpu.cfs_quota_us: {q} / {per}"
    except (OSError, ValueError):
        return None, "no cgroup cpu quota file"


def cpu_share():
    """(processes to run, affinity CPUs, quota CPUs or None, how the count was chosen): the cgroup CPU
    quota when one is set, else the affinity set capped at the 16 CPUs a one-GPU box grants per GPU
    (os.cpu_count() and the affinity set show the whole host there)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    quota, src = cgroup_cpu_quota()
    if quota is not None:
        return max(1, min(aff, int(quota))), aff, quota, f"cgroup quota ({src})"
    return min(16, aff), aff, None, f"affinity set capped at 16 ({src}: unlimited or absent)"


def cpu_baseline(players, procs, steps_per_proc):
    """The C oracle (a port of the reference engine) as single-env random rollouts, timed on this
    host BEFORE the process touches the GPU (fork-safe): a 1-core leg (one process) and an all-core
    leg (`procs` processes, one per core of the box's share)."""
    n1, w1, _, _ = _cpu_leg(players, 1, steps_per_proc)
    n, wall, per_core, eps = _cpu_leg(players, procs, steps_per_proc)
    _, aff, quota, how = cpu_share()
    return {"value": round(n / wall, 1), "unit": "env-steps/s", "cores": procs, "kind": "port",
            "one_core": round(n1 / w1, 1), "per_core_mean_all_core_leg": round(per_core, 1),
            "os_cpu_count": os.cpu_count(), "affinity_cpus": aff, "cgroup_quota_cpus": quota, "cores_source": how,
            "sample": (f"C oracle (port of engine/rules.py + envs/splendor_env.py step), {players}p, 1 env per "
                       f"process, uniform-random legal policy with autoreset: all-core leg {procs} processes x "
                       f"{steps_per_proc} env steps ({eps} episodes) = value; 1-core leg 1 process x "
                       f"{steps_per_proc} steps = one_core.  cores = processes run (cores_source says how the "
                       "count was chosen; os_cpu_count is the whole host's).  Reference Python engine: 5.4k steps/s/core, "
                       "SURVEY.md §6")}


def region_mark(name, edge, kernel=None, launches=None):
    """A timed region's edge on stderr as one JSON line with CLOCK_BOOTTIME / CLOCK_MONOTONIC stamps:
    tools/trace_timed.py picks the region's launches of `kernel` out of a rocprofv3 kernel trace of the
    same run by these (so a committed profile can be averaged over the timed launches only)."""
    rec = {"timed_region": name, "edge": edge, "boottime_ns": time.clock_gettime_ns(time.CLOCK_BOOTTIME),
           "monotonic_ns": time.monotonic_ns()}
    if kernel is not None:
        rec.update(kernel=kernel, launches=launches)
    print(json.dumps(rec), file=sys.stderr, flush=True)


def launch_spread(times):
    """min / median / max / mean of per-launch times (seconds) -> microseconds, and the median in s."""
    xs = sorted(times)
    n = len(xs)
    med = xs[n // 2] if n % 2 else 0.5 * (xs[n // 2 - 1] + xs[n // 2])
    return {"median_s": med, "us": {"min": round(xs[0] * 1e6, 2), "median": round(med * 1e6, 2),
                                    "max": round(xs[-1] * 1e6, 2), "mean": round(sum(xs) / n * 1e6, 2),
                                    "launches": n}}


def load_pmc_traffic(kernel, tables, steps_per_launch):
    """HBM bytes per launch of `kernel` on this workload from the committed rocprofv3 PMC summary
    (tools/pmc.sh -> profiles/pmc_summary.json), or (None, None)."""
    path = os.path.join(REPO, "profiles", "pmc_summary.json")
    try:
        with open(path) as f:
            e = json.load(f)["entries"].get(f"{kernel}|T{tables}|K{steps_per_launch}")
        if e and e.get("hbm_bytes_per_launch"):
            return e["hbm_bytes_per_launch"], f"{os.path.relpath(path, REPO)} ({e.get('source')})"
    except (OSError, ValueError, KeyError, AttributeError):
        pass
    return None, None


def node_fields(census, metric):
    """The JSON line's node fields from parallel.device_census: n_gpus = the
    number of DISTINCT devices the ranks ran on, ranks, the device identities and shared_device; when
    ranks share a device the metric is relabelled, as that run is a rehearsal, not a node figure."""
    shared = bool(census["shared_device"])
    if shared:
        metric = metric.replace("(whole node)", f"(shared-device rehearsal: {census['ranks']} ranks on "
                                                f"{census['devices']} GPU{'s' if census['devices'] != 1 else ''}, "
                                                "not a node figure)")
    return {"metric": metric, "n_gpus": census["devices"], "ranks": census["ranks"],
            "devices": census["identities"], "shared_device": shared}


SELFPLAY_GRAPH_STEPS = 4


def selfplay_line(dev, rank, world, N, iters, warmup, precision="fp32"):
    """BASELINE config 5 per GPU: the PPO rollout step of ppo_splendor.py:227-269 for N tables —
    the agent's fused fp32 ActorCritic (get_action_and_value: actor + critic + masked sample) and
    DualStepVectorEnv.dual_step with the reference's opponent supplier (current policy p=0.25, else
    one of 12 frozen snapshots per episode, greedy; reset after done), all weights from the
    reference checkpoint (tests/golden/ppo_splendor_latest.safetensors, fixture data), captured in a
    hipGraph.  A dual step is two env-steps.  Timed like the headline: barrier +
    synchronize around `iters` replays, max over ranks."""
    import torch
    from safetensors.torch import load_file
    from splendor_gym.fused_policy import FusedActorCritic, OpponentPool
    from splendor_gym.parallel import barrier, max_over_ranks
    from splendor_gym.policy import ActorCritic
    from splendor_gym.selfplay import DualStepVectorEnv
    ckpt = os.path.join(REPO, "tests", "golden", "ppo_splendor_latest.safetensors")

    def net():
        m = ActorCritic().to(dev).eval()
        m.load_state_dict(load_file(ckpt, device=str(dev)))
        return m

    agent = net()
    agent_k = FusedActorCritic(agent, precision=precision)
    pool = OpponentPool(agent, pool_size=12, p_current=0.25, seed=99, precision=precision)
    for _ in range(12):
        pool.add_snapshot(net())
    # the agent's sampling draws are keyed by (seed; table, ply_base): the dual step's last launch
    # advances ply_base (spl_dual_io_t.step_counter), so every captured step draws fresh actions
    ply_t = torch.zeros(1, dtype=torch.int64, device=dev)
    # the agent reads the env's compact uint8 copy of its observation (agent_obs_u8, written by the
    # opponent's step beside the int32 obs dual_step returns): a quarter of the bytes
    env = DualStepVectorEnv(N, device=dev, opponent=pool, table0=rank * N, opponent_obs=False, step_counter=ply_t,
                            agent_obs_u8=True)
    obs, info = env.reset(seed=rank * N)
    mask = info["action_mask"]
    agent_in = env.agent_obs_u8

    def iteration():
        with torch.no_grad():
            a, _, _, _ = agent_k.act(agent_in, mask, seed=1234, table0=rank * N, ply_base=ply_t)
            return env.dual_step(a)

    for _ in range(warmup):
        iteration()
    torch.cuda.synchronize(dev)
    side = torch.cuda.Stream(device=dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        iteration()
    torch.cuda.current_stream(dev).wait_stream(side)
    # SELFPLAY_GRAPH_STEPS dual steps per hipGraph (the host's replay call sits between graphs, ~8 us
    # of idle GPU per replay in the round-5 trace): every step's work is in the graph
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        for _ in range(SELFPLAY_GRAPH_STEPS):
            iteration()
    graph.replay()
    torch.cuda.synchronize(dev)
    barrier(dev)
    iters = max(SELFPLAY_GRAPH_STEPS, iters - iters % SELFPLAY_GRAPH_STEPS)
    region_mark("config5_selfplay", "start")
    t0 = time.perf_counter()
    for _ in range(iters // SELFPLAY_GRAPH_STEPS):
        graph.replay()
    torch.cuda.synchronize(dev)
    region_mark("config5_selfplay", "end")
    barrier(dev)
    el = max_over_ranks(time.perf_counter() - t0, device=dev)
    # the agent's actor + critic + masked sample (k_act32<true, true>) on its own, eager, HIP events
    # around each launch on the launch stream: its MFMA roofline
    strm = torch.cuda.current_stream(dev)
    n_act = 16
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n_act)]
    for a, b in ev:
        a.record(strm)
        b.record(strm)
    act_out = {"action": torch.empty(N, dtype=torch.int32, device=dev),
               "logprob": torch.empty(N, dtype=torch.float32, device=dev),
               "entropy": torch.empty(N, dtype=torch.float32, device=dev),
               "value": torch.empty(N, 1, dtype=torch.float32, device=dev)}
    with torch.no_grad():
        agent_k.act(agent_in, mask, seed=77, table0=rank * N, out=act_out)
        torch.cuda.synchronize(dev)
        region_mark(f"config5_actor_{precision}", "start",
                    "k_act32<true, true>" if precision == "fp32" else "k_act32h<true, true>", n_act)
        for i, (a, b) in enumerate(ev):
            a.record(strm)
            agent_k.act(agent_in, mask, seed=77, ply=i, table0=rank * N, out=act_out)
            b.record(strm)
        torch.cuda.synchronize(dev)
        region_mark(f"config5_actor_{precision}", "end")
    spread = launch_spread([a.elapsed_time(b) / 1e3 for a, b in ev])
    fa, fc = actor_critic_mfma_flop(precision)
    flop = (fa + fc) * N
    tflops = flop / spread["median_s"] / 1e12
    # the opponent pool's greedy call on its own: spl_policy_act_grouped = count +
    # place + the grouped actor over each network's full 128-table workgroups + the narrow kernel over
    # the groups' tails, eager, HIP events around each call on the launch stream, on the tables' current
    # opponents and compact rows
    oev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n_act)]
    for a, b in oev:
        a.record(strm)
        b.record(strm)
    opp_args = (env.opp_obs_u8, env.eng.mask, env.opp_group)
    opp_out = torch.empty(N, dtype=torch.int32, device=dev)
    with torch.no_grad():
        env.pool.act(*opp_args, out=opp_out)
        torch.cuda.synchronize(dev)
        region_mark(f"config5_opponent_{precision}", "start", f"k_act32{'h' if precision != 'fp32' else ''}<false, false>",
                    n_act)
        for a, b in oev:
            a.record(strm)
            env.pool.act(*opp_args, out=opp_out)
            b.record(strm)
        torch.cuda.synchronize(dev)
        region_mark(f"config5_opponent_{precision}", "end")
    ospread = launch_spread([a.elapsed_time(b) / 1e3 for a, b in oev])
    groups = torch.bincount(env.opp_group.to(torch.int64).flatten())
    full_wg = int((groups // 128).sum().item())
    tails = int(((groups % 128) > 0).sum().item())
    oflop = fa * N
    otflops = oflop / ospread["median_s"] / 1e12
    env.close()
    l1, hid = MFMA_PRODUCTS[precision]
    kname = "k_act32<true, true>" if precision == "fp32" else "k_act32h<true, true>"
    return {"metric": f"env-steps/sec (whole node), 2p self-play, on-device fp32 ActorCritic, {N} tables/GPU",
            "value": round(2 * N * world * iters / el, 1), "unit": "env-steps/s",
            "ms_per_dual_step": round(el / iters * 1e3, 4), "iters": iters,
            "precision": precision, "dtype": PRECISION_DTYPE[precision],
            "roofline": {"bound": "mfma", "achieved": round(tflops, 1), "peak": F16_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": round(tflops / F16_MFMA_PEAK_TFLOPS, 4), "kernel": kname,
                         "kernel_us": spread["us"], "flop_per_launch": flop,
                         "fp32_equivalent_tflops": round(NET_FP32_FLOP * N / spread["median_s"] / 1e12, 1),
                         "flop_note": f"16-bit MFMA work per table: actor 2*(297*256*{l1} + 256*256*{hid} + 256*45*{hid}) "
                                      f"+ critic 2*(297*256*{l1} + 256*256*{hid}) = {fa + fc} ({l1} plane products in "
                                      f"layer 1, {hid} in layers 2-3; the critic's 256->1 output on VALU); frac from the "
                                      "median of 16 eager launches (HIP events on the launch stream); "
                                      "fp32_equivalent_tflops = the network's 2 x MACs per table at that time",
                         "traffic": None},
            "opponent_roofline": {"bound": "mfma", "achieved": round(otflops, 1), "peak": F16_MFMA_PEAK_TFLOPS,
                                  "unit": "TFLOP/s", "frac": round(otflops / F16_MFMA_PEAK_TFLOPS, 4),
                                  "kernel": f"spl_policy_act_grouped: k_group_count + k_group_place + "
                                            f"{kname.replace('true, true', 'false, false')} + k_act32_narrow",
                                  "call_us": ospread["us"], "flop_per_call": oflop,
                                  "networks": int((groups > 0).sum().item()), "full_workgroups": full_wg,
                                  "tail_groups": tails,
                                  "flop_note": f"16-bit MFMA work of the greedy actor per table: 2*(297*256*{l1} + "
                                               f"256*256*{hid} + 256*45*{hid}) = {fa} (no critic); frac from the median "
                                               f"of {n_act} eager calls (HIP events on the launch stream around the whole "
                                               "grouped call, its two small grouping launches included)"},
            "config": {"workload": f"BASELINE config 5 per GPU: ActorCritic.get_action_and_value (fused, precision "
                                   f"{precision}) + DualStepVectorEnv.dual_step, opponent pool (current p=0.25 else 1 of "
                                   "12 frozen snapshots per episode, greedy, same precision), reset after done; hipGraph replays "
                                   f"of {SELFPLAY_GRAPH_STEPS} dual steps; the agent reads the compact uint8 copy of its "
                                   "observation that the opponent's step writes beside the int32 rows",
                       "tables_per_gpu": N, "weights": "reference checkpoint runs/ppo_splendor/ppo_splendor_latest.pt"}}


def caller_path_line(n_envs=16, iters=150, warmup=10):
    """The UNCHANGED ppo_splendor.py rollout loop: `n_envs` envs built by
    training_utils.make_env (DualStepNativeWrapper(SplendorEnv()) with the random opponent, each reset
    with its own seed), driven one env at a time in Python exactly as ppo_splendor.py:235-269 does —
    env.dual_step(action), env.reset() after done.  The agent's actions are uniform over each env's
    legal mask (numpy), so the line times the env path alone, not the torch agent.  Every
    SplendorEnv.step here is a one-table spl_step launch that reads its action from and writes its
    ~1.3 KB of outputs to pinned host memory, then one stream synchronisation; the line reports env-steps/s (every SplendorEnv.step call: agent, opponent and
    the openings after resets) and the time per SplendorEnv.step."""
    import numpy as np
    from training_utils import make_env
    np.random.seed(0)
    envs = [make_env(1000 + i, use_dual_player=True)() for i in range(n_envs)]
    clock = {"n": 0, "s": 0.0}
    for w in envs:  # time every SplendorEnv.step (launch + stream synchronisation)
        inner = w.env
        raw = inner.step

        def timed(action, raw=raw):
            t = time.perf_counter()
            r = raw(action)
            clock["s"] += time.perf_counter() - t
            clock["n"] += 1
            return r
        inner.step = timed
    masks = [w.env.legal_mask() for w in envs]
    rng = np.random.default_rng(1)

    def loop(k):
        for _ in range(k):
            for i, w in enumerate(envs):
                legal = np.flatnonzero(masks[i])
                a = int(rng.choice(legal)) if len(legal) else 0
                _, _, _, _, done, info = w.dual_step(a)
                if done:
                    _, info = w.reset()
                masks[i] = info["action_mask"]

    loop(warmup)
    clock.update(n=0, s=0.0)
    t0 = time.perf_counter()
    loop(iters)
    el = time.perf_counter() - t0
    steps = clock["n"]
    return {"metric": f"env-steps/sec, unchanged ppo_splendor.py loop: {n_envs} DualStepNativeWrapper(SplendorEnv()) "
                      "stepped one at a time from Python",
            "value": round(steps / el, 1), "unit": "env-steps/s", "env_steps": steps, "loop_iterations": iters,
            "us_per_splendorenv_step": round(clock["s"] / max(1, steps) * 1e6, 2),
            "us_per_dual_step": round(el / (iters * n_envs) * 1e6, 2),
            "host_share": round(1.0 - clock["s"] / el, 4),
            "note": "host-bound: one launch + one stream synchronisation per SplendorEnv.step; the batched "
                    "DualStepVectorEnv (config5_selfplay) steps every table in one launch; agent forward excluded",
            "config": {"workload": "ppo_splendor.py:151-159,235-269 rollout loop shape, random legal agent actions, "
                                   "random_opponent", "envs": n_envs}}


def partner_stats(lib, clear=False):
    """The six-wave dealer's partner hand-off counters (spl_debug_partner_stats; synchronises)."""
    import ctypes
    st = (ctypes.c_uint64 * 2)()
    if lib.spl_debug_partner_stats(st, 1 if clear else 0) != 0:
        return None
    return {"stored_by_partner": int(st[0]), "claimed_back": int(st[1])}


def c4_share_line(dev, rank, world, T, launches, warmup, pipeline=True, partner_lead=None):
    """BASELINE config 4's per-GPU share (262 144 4-player tables over 8 GPUs = 32 768 per GPU) on
    this rank: the same per-step rollout store as the headline (spl_rollout, 128 steps per launch,
    every step's obs/mask/reward/terminated/flags/winner into [128, T, ...]), `launches` launches
    timed with HIP events around each (after `warmup`), barrier + synchronize around the timed
    region, max over ranks; roofline bytes as the headline's."""
    import torch
    from splendor_gym import _native
    from splendor_gym.device import Engine
    from splendor_gym.parallel import barrier, max_over_ranks
    P, K = 4, ROLLOUT_K
    table0 = rank * T
    eng = Engine(T, P, device=dev, refill_period=REFILL_EVERY[P], table0=table0, pipeline=pipeline,
                 partner_lead=partner_lead)
    eng.reset(seeds=range(table0, table0 + T))
    out = dict(obs=torch.zeros((K, T, 297), dtype=torch.int32, device=dev),
               mask=torch.zeros((K, T, 45), dtype=torch.int8, device=dev),
               reward=torch.zeros((K, T), dtype=torch.float32, device=dev),
               terminated=torch.zeros((K, T), dtype=torch.uint8, device=dev),
               flags=torch.zeros((K, T), dtype=torch.uint8, device=dev),
               winner=torch.zeros((K, T), dtype=torch.int8, device=dev),
               final_obs=torch.zeros((K, T, 297), dtype=torch.int32, device=dev))
    acts = [torch.zeros(T, dtype=torch.int32, device=dev) for _ in range(2)]
    eng.sample_uniform(out=acts[0], seed=3, ply=0)
    ep_cnt = torch.zeros(T, dtype=torch.int32, device=dev)
    ply = 1

    def launch(i):
        nonlocal ply
        eng.rollout(K, actions=acts[i & 1], next_actions=acts[(i & 1) ^ 1], policy_seed=3, ply=ply, out=out,
                    ep_count=ep_cnt)
        ply += K

    for i in range(warmup):
        launch(i)
    strm = torch.cuda.current_stream(dev)
    ev0 = [torch.cuda.Event(enable_timing=True) for _ in range(launches)]
    ev1 = [torch.cuda.Event(enable_timing=True) for _ in range(launches)]
    for e in ev0 + ev1:  # created on first record, outside the timed region
        e.record(strm)
    torch.cuda.synchronize(dev)
    eps0 = int(ep_cnt.sum().item())
    partner_stats(eng.lib, clear=True)
    barrier(dev)
    region_mark("config4_share", "start", eng.rollout_kernel_name(per_step=True), launches)
    t0 = time.perf_counter()
    for i in range(launches):
        ev0[i].record(strm)
        launch(warmup + i)
        ev1[i].record(strm)
    torch.cuda.synchronize(dev)
    region_mark("config4_share", "end")
    barrier(dev)
    el = max_over_ranks(time.perf_counter() - t0, device=dev)
    times = [ev0[i].elapsed_time(ev1[i]) / 1e3 for i in range(launches)]
    launch_s = sum(times) / launches
    spread = launch_spread(times)
    term = (int(ep_cnt.sum().item()) - eps0) / launches
    algo = (2 * STATE_BYTES[P] + 8) * T + OUT_BYTES * T * K + OBS_ROW * term
    name = eng.rollout_kernel_name(per_step=True)
    traffic, src = load_pmc_traffic(name, T, K)
    # the dealer kernel's hand-off faults (spl_ctx_faults) and error flags of the last launch's steps
    faults = eng.faults()
    handoffs = partner_stats(eng.lib)
    bad = int(((out["flags"] & (_native.F_OOB | _native.F_AFTER_TERMINAL | _native.F_FAULT)) != 0).sum().item())
    eng.close()
    achieved = algo / spread["median_s"] / 1e9
    return {"metric": f"env-steps/sec (whole node), 4p {T} tables/GPU (BASELINE config 4's per-GPU share)",
            "value": round(T * world * K * launches / el, 1), "unit": "env-steps/s",
            "ms_per_step": round(el / (K * launches) * 1e3, 4), "steps": K * launches, "warmup_launches": warmup,
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "kernel": name, "steps_per_launch": K,
                         "kernel_avg_us": round(launch_s * 1e6, 2), "kernel_us": spread["us"],
                         "kernel_timing": f"HIP events around each of {launches} eager launches in the timed region; "
                                          "frac from the median launch",
                         "algo_bytes_per_launch": round(algo),
                         "algo_bytes_note": f"as the headline's, 4 players ({term:.0f} terminal rows per launch)",
                         "traffic": traffic, "traffic_source": src,
                         "traffic_over_algo": None if traffic is None else round(traffic / algo, 4)},
            "error_flags": bad, "launch_faults": faults,
            "partner_handoffs": None if handoffs is None else dict(handoffs, launches=launches,
                                                                   row_blocks_per_launch=K * T // 64),
            "config": {"workload": "4-player SplendorEnv.step, device uniform-random policy, same-step autoreset, "
                                   "per-step rollout store [128, T, ...]", "tables_per_gpu": T, "players": P}}


STEP_SHAPE_SUFFIX = {0: "ws", 1: "wst", 2: "wso"}


def step_shape(mode, tables, cus=None):
    """spl_step's kernel shape for `tables` tables of full int32 outputs: the forced mode, or the library's
    auto rule (spl_engine.hip spl_step: three waves up to three 64-table workgroups per CU, else two)."""
    if mode != "auto":
        return int(mode)
    if cus is None:
        import torch
        cus = torch.cuda.get_device_properties(torch.cuda.current_device()).multi_processor_count
    return 1 if -(-int(tables) // 64) <= 3 * int(cus) else 0


def self_launch(n, argv, device_count=None):
    """`python bench.py --gpus N` without a launcher: N ranks of this script on this node, one per GPU
    (parallel.launch_local_ranks; rank r drives cuda:r, rank 0 prints the JSON line).  This process
    only counts the devices (torch.cuda.device_count() creates no HIP context) and waits; it exits
    with the first failing rank's status.  Fewer than N devices: exit 2 with a message, nothing run.
    No CPU baseline at N > 1 (it is reported at N = 1 only).  SPLENDOR_SHARED_DEVICE_REHEARSAL=1 lets N ranks share
    fewer GPUs (with SPLENDOR_DIST_BACKEND=gloo): the line then says "shared-device rehearsal", not a node figure."""
    if device_count is None:
        import torch
        device_count = torch.cuda.device_count()
    from splendor_gym.parallel import REHEARSAL_ENV
    if device_count < n and os.environ.get(REHEARSAL_ENV) != "1":
        print(f"bench.py --gpus {n}: this node shows {device_count} GPU(s); a run on {n} GPUs needs {n} "
              f"(no figure reported)", file=sys.stderr, flush=True)
        return 2
    if device_count < 1:
        print(f"bench.py --gpus {n}: no GPU visible", file=sys.stderr, flush=True)
        return 2
    from splendor_gym.parallel import launch_local_ranks
    return launch_local_ranks(n, [sys.executable, os.path.abspath(__file__), *argv])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1024)
    ap.add_argument("--warmup", type=int, default=128)
    ap.add_argument("--tables", type=int, default=65536, help="tables per GPU")
    ap.add_argument("--players", type=int, default=2)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-procs", type=int, default=0, help="0 = the cgroup CPU quota, else min(16, affinity CPUs)")
    ap.add_argument("--cpu-steps", type=int, default=1_000_000, help="env steps per CPU process")
    ap.add_argument("--graph-steps", type=int, default=128,
                    help="step mode: steps per captured HIP graph (rounded to whole plan units); 0 = eager")
    ap.add_argument("--mode", choices=("step", "rollout"), default="rollout",
                    help="rollout: one spl_rollout launch per "
                         f"{ROLLOUT_K} env steps; step: one spl_step launch per env step (same trajectories "
                         "and per-step outputs, tests/test_gpu_parity.py::test_rollout_equals_step_chain)")
    ap.add_argument("--only", action="store_true", help="measure only --mode's headline variant")
    ap.add_argument("--outputs", choices=("store", "inplace"), default="store",
                    help="rollout mode: per-step blocks of a [K, T, ...] rollout store (headline) or every "
                         "step into the same block (L3-resident; labelled in_place_l3)")
    ap.add_argument("--rollout-k", type=int, default=ROLLOUT_K, help="env steps per spl_rollout launch")
    ap.add_argument("--refill-every", type=int, default=0, help="0 = per player count (64/32/16)")
    ap.add_argument("--refill", choices=("fused", "separate"), default="fused",
                    help="rollout mode: due pool refills run inside the spl_rollout launch (fused) or as a "
                         "spl_refill launch after it (step mode always launches spl_refill)")
    ap.add_argument("--pipeline", choices=("auto", "always", "half", "off", "dealer", "dealer2", "quad"), default="auto",
                    help="rollout mode: two-wave pipelined kernel (auto: 32 or 64 tables per workgroup by grid "
                         "size; always: 64; half: 32) vs one wave per 64 tables (off)")
    ap.add_argument("--sp-tables", type=int, default=65536,
                    help="tables per GPU of the config-5 self-play line (0 = skip it)")
    ap.add_argument("--sp-iters", type=int, default=64, help="timed dual steps of the config-5 line")
    ap.add_argument("--caller-envs", type=int, default=16,
                    help="envs of the unchanged ppo_splendor.py caller-path line (0 = skip it)")
    ap.add_argument("--c4-tables", type=int, default=32768,
                    help="tables per GPU of the config-4 share line (4 players; 0 = skip)")
    ap.add_argument("--c4-pipeline", default=True, type=lambda v: {"auto": True}.get(v, v),
                    help="rollout kernel of the config-4 share line: auto (default), dealer, dealer2, always, half")
    ap.add_argument("--delegation", type=int, default=0,
                    help="rollout store: every n-th step the odd-XCC workgroups' rows are stored by their "
                         "even-XCC partners (0 = off, the library default: a 1.5 %% gain, "
                         "profiles/r03/deleg_ab_r03a.txt)")
    ap.add_argument("--step-tail", choices=("auto", "0", "1", "2"), default="auto",
                    help="spl_step kernel shape: auto (the library's choice by grid size), 0 two waves, 1 three waves "
                         "(a tail wave takes the legal mask off the rules wave), 2 two waves with the output wave "
                         "taking it between its row stores; same results")
    ap.add_argument("--partner-lead", type=int, default=None,
                    help="rollout store (six-wave dealer and quad kernels): a team this many steps behind its "
                         "neighbouring-XCC partner hands it whole steps of rows (library default 0 = off; "
                         "-1 = whenever a slot is free)")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(self_launch(args.gpus, sys.argv[1:]))

    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    rank_env = int(os.environ.get("RANK", "0"))
    cpu = None
    if world_env == 1 and rank_env == 0 and not args.no_cpu_baseline:
        procs = args.cpu_procs or cpu_share()[0]
        cpu = cpu_baseline(args.players, procs, args.cpu_steps)

    import torch
    from splendor_gym import _native
    from splendor_gym.device import Engine
    from splendor_gym.parallel import (barrier, device_census, device_identity, gather_returns, init_distributed,
                                       local_device, max_over_ranks, require_distinct_devices)

    rank, world, local = init_distributed()
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    dev = local_device(local)
    torch.cuda.set_device(dev)
    # which physical GPU each rank drives: n_gpus counts distinct devices, not ranks
    census = device_census(device_identity(dev))
    err = require_distinct_devices(census, world)
    if err is not None:  # self-launched ranks sharing a card: not an N-GPU run
        if rank == 0:
            print(f"bench.py --gpus {args.gpus}: {err}", file=sys.stderr, flush=True)
        sys.exit(3)
    if census["shared_device"] and rank == 0:
        print(f"warning: {census['ranks']} ranks share {census['devices']} device(s): {census['identities']}",
              file=sys.stderr)
    T, P = args.tables, args.players
    R = args.refill_every or REFILL_EVERY[P]
    RK = args.rollout_k
    table0 = rank * T
    pipe = {"auto": True, "always": "always", "half": "half", "off": False, "dealer": "dealer",
            "dealer2": "dealer2", "quad": "quad"}[args.pipeline]
    eng = Engine(T, P, device=dev, refill_period=R, table0=table0, refill_fused=args.refill == "fused",
                 pipeline=pipe, delegation=args.delegation, partner_lead=args.partner_lead,
                 step_tail=None if args.step_tail == "auto" else int(args.step_tail))
    eng.reset(seeds=range(table0, table0 + T))
    lib = eng.lib
    buf = [torch.zeros(T, dtype=torch.int32, device=dev) for _ in range(2)]
    eng.sample_uniform(out=buf[0], seed=args.seed, ply=0)
    ep_ret = torch.zeros(T, dtype=torch.float32, device=dev)
    ep_cnt = torch.zeros(T, dtype=torch.int32, device=dev)
    ply_base = torch.zeros(1, dtype=torch.int64, device=dev)  # policy counter base (graph replays advance it)

    # rollout store: step k of a launch writes block k (obs/final_obs 5 GB each at 65536 tables)
    store = None

    def get_store():
        nonlocal store
        if store is None:
            # zero-filled once, so the first launches do not pay first-touch costs that the timed
            # ones never see (a rocprofv3 row then averages like the timed launches)
            store = dict(obs=torch.zeros((RK, T, 297), dtype=torch.int32, device=dev),
                         mask=torch.zeros((RK, T, 45), dtype=torch.int8, device=dev),
                         reward=torch.zeros((RK, T), dtype=torch.float32, device=dev),
                         terminated=torch.zeros((RK, T), dtype=torch.uint8, device=dev),
                         flags=torch.zeros((RK, T), dtype=torch.uint8, device=dev),
                         winner=torch.zeros((RK, T), dtype=torch.int8, device=dev),
                         final_obs=torch.zeros((RK, T, 297), dtype=torch.int32, device=dev))
        return store

    def mkargs(a_in, a_out, bufs):
        return _native.StepArgs(actions=a_in.data_ptr(), obs=bufs["obs"].data_ptr(), mask=bufs["mask"].data_ptr(),
                                reward=bufs["reward"].data_ptr(), terminated=bufs["terminated"].data_ptr(),
                                flags=bufs["flags"].data_ptr(), winner=bufs["winner"].data_ptr(),
                                final_obs=bufs["final_obs"].data_ptr(), autoreset=1, next_actions=a_out.data_ptr(),
                                ply_base=ply_base.data_ptr(), policy_seed=args.seed, ply=0, table0=table0,
                                ep_return=ep_ret.data_ptr(), ep_count=ep_cnt.data_ptr())

    eng_bufs = dict(obs=eng.obs, mask=eng.mask, reward=eng.reward, terminated=eng.terminated, flags=eng.flags,
                    winner=eng.winner, final_obs=eng.final_obs)
    ctx, desc = eng.ctx, ctypes.byref(eng.desc)
    stream = eng.stream()

    def step_args(variant):
        """The two alternating argument blocks of a variant (built outside any timed region)."""
        bufs = get_store() if variant == "rollout_store" else eng_bufs
        return [mkargs(buf[0], buf[1], bufs), mkargs(buf[1], buf[0], bufs)]

    def run(variant, k0, k1, strm, ev=None, sargs=None):
        """Env steps k0..k1-1 (ply k+1 relative to ply_base).  variant "step": one spl_step launch
        per step; "rollout_store"/"rollout_inplace": one spl_rollout launch per RK steps with
        per-step blocks / in place.  Refills every R steps are issued by the library."""
        per = 1 if variant == "step" else RK
        sargs = sargs or step_args(variant)
        for i, k in enumerate(range(k0, k1, per)):
            sa = sargs[(k // per) & 1]
            sa.ply = k + 1
            if ev is not None:
                ev[0][i].record()
            if variant == "step":
                _native.check(lib, lib.spl_step(ctx, desc, ctypes.byref(sa), strm))
            else:
                _native.check(lib, lib.spl_rollout(ctx, desc, ctypes.byref(sa), RK,
                                                   1 if variant == "rollout_store" else 0, strm))
            if ev is not None:
                ev[1][i].record()

    def kernel_name(variant):
        """The kernel the variant launches, as rocprofv3 names it (one name per instantiation)."""
        if variant == "step":  # spl_step's shape (include/splendor_amd.h spl_ctx_set_step_tail), as the library picks it
            return f"k_step_{STEP_SHAPE_SUFFIX[step_shape(args.step_tail, T)]}_{P}p"
        return eng.rollout_kernel_name(per_step=variant == "rollout_store")

    def events(n):
        return ([torch.cuda.Event(enable_timing=True) for _ in range(n)],
                [torch.cuda.Event(enable_timing=True) for _ in range(n)])

    def measure(variant, k_base):
        """Warm up, time K steps; returns the timing record.  Steps are numbered from k_base so
        every measurement continues the same trajectories with fresh policy counters."""
        plan = step_plan("step" if variant == "step" else "rollout", args.steps, args.warmup, R, RK,
                         args.graph_steps)
        K, W, G, per = plan["K"], plan["W"], plan["G"], plan["per"]
        # warm-up: W steps, eager (also allocates the rollout store outside the timed region)
        ply_base.fill_(k_base)
        run(variant, 0, W, stream)
        graph = None
        how = "eager launches, HIP events around each launch"
        if G > 0:
            try:
                torch.cuda.synchronize(dev)
                ply_base.fill_(k_base + W)
                graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(graph):
                    run(variant, 0, G, ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream))
                    ply_base.add_(G)
                how = f"hipGraph replays of {G} steps"
            except Exception as exc:  # capture unsupported: time eager launches instead
                print(f"graph capture failed ({exc}); timing eager launches", file=sys.stderr)
                graph, G = None, 0
        warm_replays = 0
        if graph is not None:  # one untimed replay: the graph's first launch is not part of the measurement
            graph.replay()
            warm_replays = 1
        torch.cuda.synchronize(dev)
        eps0 = int(ep_cnt.sum().item())
        barrier(dev)
        ev = events(K // G) if graph is not None else events(K // per)
        sargs = step_args(variant)
        if graph is None:
            ply_base.fill_(k_base + W)
        for e in ev[0] + ev[1]:  # the HIP events are created on first record: outside the timed region
            e.record()
        torch.cuda.synchronize(dev)
        region_mark(variant, "start", kernel_name(variant), K // per)
        t0 = time.perf_counter()
        if graph is not None:
            # recorded on the replay stream around each replay, not as graph nodes
            for i in range(K // G):
                ev[0][i].record()
                graph.replay()
                ev[1][i].record()
        else:
            run(variant, 0, K, stream, ev, sargs)
        t_enq = time.perf_counter()
        torch.cuda.synchronize(dev)
        t_sync = time.perf_counter()
        region_mark(variant, "end")
        barrier(dev)
        elapsed = max_over_ranks(time.perf_counter() - t0, device=dev)
        span = ev[0][0].elapsed_time(ev[1][-1]) / 1e3
        print(f"[{variant}] timed region: wall {(t_sync - t0) * 1e3:.3f} ms (host enqueue "
              f"{(t_enq - t0) * 1e3:.3f} ms), GPU span first->last event {span * 1e3:.3f} ms", file=sys.stderr)
        terminations = int(ep_cnt.sum().item()) - eps0
        kt = "HIP events around each launch in the timed region"
        k_next = k_base + W + warm_replays * G + K + 1
        eager_s = None
        if graph is not None:
            # ROCm rejects timing events as graph nodes ("External events are disallowed"), so the
            # per-launch time is each replay's event interval over its G launches (the graph's
            # inter-kernel gaps included); HIP events around each launch of an eager window of the
            # same loop, right after the timed replays, are reported beside it (they also bracket
            # the host dispatch latency of a ~20 us kernel).
            times = [ev[0][i].elapsed_time(ev[1][i]) / 1e3 / (G // per) for i in range(len(ev[0]))]
            launch_s = sum(times) / len(times)
            kt = f"HIP events around each of {K // G} hipGraph replays ({G // per} launches each) in the timed region"
            nwin = plan["unit"] * max(1, -(-64 // plan["unit"]))
            ev = events(nwin // per)
            ply_base.fill_(k_next)
            run(variant, 0, nwin, stream, ev)
            torch.cuda.synchronize(dev)
            eager_s = sum(ev[0][i].elapsed_time(ev[1][i]) for i in range(len(ev[0]))) / len(ev[0]) / 1e3
            k_next += nwin + 1
        else:
            times = [ev[0][i].elapsed_time(ev[1][i]) / 1e3 for i in range(len(ev[0]))]
            launch_s = sum(times) / len(times)
        return {"variant": variant, "plan": plan, "elapsed": elapsed, "launch_s": launch_s, "times": times, "how": how,
                "kernel_timing": kt, "terminations": terminations, "k_next": k_next, "eager_s": eager_s}

    headline = "step" if args.mode == "step" else ("rollout_store" if args.outputs == "store" else "rollout_inplace")
    variants = [headline]
    if not args.only:
        variants += [v for v in ("rollout_store", "rollout_inplace", "step") if v != headline]
    recs, k_next = {}, 0
    handoffs = None
    for v in variants:
        if v == "rollout_store":
            partner_stats(lib, clear=True)
        recs[v] = measure(v, k_next)
        k_next = recs[v]["k_next"]
        if v == "rollout_store" and headline == "rollout_store":  # this line's hand-offs (warm-up included)
            handoffs = partner_stats(lib)
    sp = sp2 = None
    if args.sp_tables > 0 and not args.only:
        sp = selfplay_line(dev, rank, world, args.sp_tables, args.sp_iters, warmup=8, precision="fp32")
        sp2 = selfplay_line(dev, rank, world, args.sp_tables, args.sp_iters, warmup=8, precision="fp32_f16x2")
    c4 = None
    if args.c4_tables > 0 and not args.only and args.players == 2:
        c4 = c4_share_line(dev, rank, world, args.c4_tables, launches=8, warmup=2, pipeline=args.c4_pipeline,
                           partner_lead=args.partner_lead)
    caller = None
    if args.caller_envs > 0 and not args.only and rank == 0 and args.players == 2:
        caller = caller_path_line(args.caller_envs)
    # correctness canaries on the measured run: no error flags, episodes completed
    errs = _native.F_OOB | _native.F_AFTER_TERMINAL | _native.F_RNG_LIMIT | _native.F_FAULT
    bad = int(((eng.flags & errs) != 0).sum().item())
    if store is not None:  # every step of the last rollout-store launch
        bad += int(((store["flags"] & errs) != 0).sum().item())
    faults = eng.faults()
    rets, cnts = gather_returns(ep_ret, ep_cnt.to(torch.int64), n_global=T * world)
    episodes = int(cnts.sum().item())

    def summary(rec):
        v, plan = rec["variant"], rec["plan"]
        K, per = plan["K"], plan["per"]
        launches = K // per
        if v == "step":
            algo = STEP_ALGO_BYTES[P] * T
            algo_note = (f"{STEP_ALGO_BYTES[P]} B per table-step (SURVEY.md §8d: 2*S_P + obs + mask + action + reward + "
                         f"terminated = {STEP_ALGO_BYTES[P] - LEGAL_CACHE_BYTES}, + {LEGAL_CACHE_BYTES} B of legal-mask cache)")
        else:
            # state read+write once per launch, first/next actions, per-step outputs, terminal rows
            term_per_launch = rec["terminations"] / launches
            algo = (2 * STATE_BYTES[P] + 8) * T + OUT_BYTES * T * per + OBS_ROW * term_per_launch
            algo_note = (f"2*S_P/{per} + {OUT_BYTES} B per table-step (obs 1188 + mask 45 + reward 4 + terminated/flags/"
                         f"winner 3) + 8 B/table of actions per launch + 1188 B per terminal row "
                         f"({term_per_launch:.0f} per launch, counted in the timed region)")
        spread = launch_spread(rec["times"])
        achieved = algo / spread["median_s"] / 1e9  # frac from the median launch
        if v == "rollout_inplace":
            # every step overwrites one ~81 MB block that stays in the 256 MiB Infinity Cache: not an
            # HBM figure, so no HBM fraction
            bound = {"bound": "l3", "achieved": round(achieved, 1), "peak": None, "unit": "GB/s", "frac": None,
                     "bound_note": "L3-resident output block (MALL): achieved is algorithmic bytes / median launch, "
                                   "no HBM fraction"}
        else:
            bound = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "frac_of_achievable": round(achieved / HBM_ACHIEVABLE_GBS, 4)}
        return {"variant": v, "value": round(T * world * K / rec["elapsed"], 1),
                "steps": K, "ms_per_step": round(rec["elapsed"] / K * 1e3, 4),
                "roofline": {**bound,
                             "kernel": kernel_name(v), "steps_per_launch": per,
                             "kernel_avg_us": round(rec["launch_s"] * 1e6, 2),
                             "kernel_us": spread["us"],
                             "kernel_timing": rec["kernel_timing"] + "; frac from the median launch",
                             **({} if rec["eager_s"] is None else
                                {"eager_launch_us": round(rec["eager_s"] * 1e6, 2)}),
                             "algo_bytes_per_launch": round(algo),
                             "algo_bytes_note": algo_note},
                "launch": rec["how"], "plan": plan}

    def with_traffic(s):
        """The variant's summary with the committed PMC HBM bytes per launch of its kernel."""
        traffic, traffic_src = load_pmc_traffic(s["roofline"]["kernel"], T, s["plan"]["per"])
        s["roofline"].update(traffic=traffic, traffic_source=traffic_src,
                             traffic_over_algo=None if traffic is None
                             else round(traffic / s["roofline"]["algo_bytes_per_launch"], 4))
        return s

    if rank == 0:
        main_s = with_traffic(summary(recs[headline]))
        roof = main_s["roofline"]
        plan = main_s["plan"]
        node = node_fields(census, f"env-steps/sec (whole node), {P}p {T} tables/GPU")
        out = {
            "metric": node.pop("metric"),
            "value": main_s["value"],
            "unit": "env-steps/s",
            **node,
            "steps": plan["K"],
            "warmup": plan["W"],
            "ms_per_step": main_s["ms_per_step"],
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic: seeded deals (table id = env seed), device uniform-random legal policy",
            "config": {"workload": f"{P}-player SplendorEnv.step x {T} tables per GPU, legal mask + uniform-random "
                                   "policy, same-step autoreset, obs int32[297] + mask int8[45] per table-step"
                                   + (" into a per-step rollout store" if headline == "rollout_store" else ""),
                       "tables_per_gpu": T, "players": P, "parallelism": f"table-sharded x{world}",
                       "refill_every": R, "refill": args.refill if headline != "step" else "separate",
                       "pipeline": args.pipeline, "rollout_steps_per_launch": RK, "variant": headline,
                       "delegation": args.delegation,
                       "launch": main_s["launch"], "requested_steps": plan["requested_steps"],
                       "requested_warmup": plan["requested_warmup"],
                       "step_rounding": f"steps/warmup rounded up to whole units of {plan['unit']} (step_plan)"},
            "roofline": roof,
            "cpu_baseline": cpu,
            "episodes": episodes,
            "mean_final_reward_p0": round(float(rets.sum().item()) / max(1, episodes), 4),
            "error_flags": bad,
            "launch_faults": faults,
        }
        if handoffs is not None:  # the headline's partner hand-offs (its warm-up and timed launches)
            out["partner_handoffs"] = dict(handoffs, row_blocks_per_launch=RK * T // 64)
        for v in variants[1:]:
            s = with_traffic(summary(recs[v]))
            s.pop("plan")
            out["in_place_l3" if v == "rollout_inplace" else ("other_mode" if v == "step" else v)] = s
        if caller is not None:
            out["caller_path"] = caller
        for key, line in (("config5_selfplay", sp), ("config5_selfplay_f16x2", sp2), ("config4_share", c4)):
            if line is not None:
                line["metric"] = node_fields(census, line["metric"])["metric"]
                out[key] = line
        print(json.dumps(out))
    eng.close()
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
