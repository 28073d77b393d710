"""Step mode (one spl_step launch per env step) as C independent chains over disjoint table ranges.

    python tools/bench_step_chains.py [--tables 65536] [--chains 1,2,4] [--graph-steps 128] [--replays 8]

All the tables' step launches in one chain run in lockstep: every workgroup does its rules (~8 us), then
the whole chip stores the 78 MB of observation rows (~12.7 us), and nothing overlaps inside a launch
(DESIGN.md §10 "Step mode: the floor").  Tables are independent, so the same env steps can be issued as
C chains of spl_step over T/C tables each (C engines whose global ids are contiguous ranges: table0 =
c*T/C — the shard invariance of test_sharded_equals_whole makes their trajectories those of one engine
of T tables), each chain on its own stream, captured as C branches of one hipGraph of G steps.  Within a
chain the launches stay ordered; between chains nothing is, so one chain's rules can run while another
chain's rows drain.  Per env step (all T tables) = replay time / G.  Every chain uses the bench's
step-mode arguments (device uniform-random policy fused into the step, same-step autoreset, final
observations, refills every 64 steps issued by the library inside the graph)."""
import argparse
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "splendor-gym_amd"))


def run(T, C, G, replays, warm, seed=0, eager=False, offset_cycles=0):
    import torch
    from splendor_gym import _native
    from splendor_gym.device import Engine
    dev = torch.device("cuda", 0)
    n = T // C
    chains = []
    for c in range(C):
        e = Engine(n, 2, device=dev, refill_period=64, table0=c * n)
        e.reset(seeds=range(c * n, (c + 1) * n))
        acts = [torch.zeros(n, dtype=torch.int32, device=dev) for _ in range(2)]
        e.sample_uniform(out=acts[0], seed=seed, ply=0)
        ply_base = torch.zeros(1, dtype=torch.int64, device=dev)

        def mk(a_in, a_out, e=e, ply_base=ply_base, c=c):
            return _native.StepArgs(actions=a_in.data_ptr(), obs=e.obs.data_ptr(), mask=e.mask.data_ptr(),
                                    reward=e.reward.data_ptr(), terminated=e.terminated.data_ptr(),
                                    flags=e.flags.data_ptr(), winner=e.winner.data_ptr(),
                                    final_obs=e.final_obs.data_ptr(), autoreset=1, next_actions=a_out.data_ptr(),
                                    ply_base=ply_base.data_ptr(), policy_seed=seed, ply=0, table0=c * n)
        chains.append(dict(eng=e, args=[mk(acts[0], acts[1]), mk(acts[1], acts[0])], ply_base=ply_base, acts=acts))
    main = torch.cuda.current_stream(dev)
    side = [torch.cuda.Stream(device=dev) for _ in range(C - 1)]

    def issue(strms, steps):
        for c, ch in enumerate(chains):
            s = strms[c]
            h = ctypes.c_void_p(s.cuda_stream)
            e = ch["eng"]
            for k in range(steps):
                sa = ch["args"][k & 1]
                sa.ply = k + 1
                _native.check(e.lib, e.lib.spl_step(e.ctx, ctypes.byref(e.desc), ctypes.byref(sa), h))
            with torch.cuda.stream(s):
                ch["ply_base"].add_(steps)

    # eager warm-up on the capture streams' pattern, then capture
    issue([main] * C, G)
    torch.cuda.synchronize(dev)
    if eager:  # eager launches, chain c on stream c, issued step by step across the chains
        strms = [main] + side
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ends = [torch.cuda.Event() for _ in strms]
        per = []
        for rep in range(warm + replays):
            ev0.record(main)
            for c, s_ in enumerate(side, start=1):
                s_.wait_event(ev0)
                if offset_cycles:  # chain c starts c x offset later: its rules phases fall into chain 0's stores
                    with torch.cuda.stream(s_):
                        torch.cuda._sleep(int(c * offset_cycles))
            for k in range(G):
                for c, ch in enumerate(chains):
                    e = ch["eng"]
                    sa = ch["args"][k & 1]
                    sa.ply = k + 1
                    _native.check(e.lib, e.lib.spl_step(e.ctx, ctypes.byref(e.desc), ctypes.byref(sa),
                                                        ctypes.c_void_p(strms[c].cuda_stream)))
            for c, ch in enumerate(chains):
                with torch.cuda.stream(strms[c]):
                    ch["ply_base"].add_(G)
            for s_, en in zip(side, ends[1:]):
                en.record(s_)
                main.wait_event(en)
            ev1.record(main)
            torch.cuda.synchronize(dev)
            if rep >= warm:
                per.append(ev0.elapsed_time(ev1) * 1e3 / G)
        per.sort()
        errs = _native.F_OOB | _native.F_AFTER_TERMINAL | _native.F_RNG_LIMIT | _native.F_FAULT
        bad = sum(int(((ch["eng"].flags & errs) != 0).sum().item()) for ch in chains)
        for ch in chains:
            ch["eng"].close()
        return {"tables": T, "chains": C, "mode": "eager", "offset_cycles": offset_cycles, "tables_per_chain": n,
                "steps": G, "reps": replays,
                "us_per_env_step": {"min": round(per[0], 3), "median": round(per[len(per) // 2], 3), "max": round(per[-1], 3)},
                "env_steps_per_s": round(T / (per[len(per) // 2] * 1e-6), 1), "error_flags": bad}
    g = torch.cuda.CUDAGraph()
    cap = torch.cuda.Stream(device=dev)
    cap.wait_stream(main)
    with torch.cuda.stream(cap):
        with torch.cuda.graph(g, stream=cap):
            for s in side:
                s.wait_stream(cap)
            issue([cap] + side, G)
            for s in side:
                cap.wait_stream(s)
    torch.cuda.synchronize(dev)
    for _ in range(warm):
        g.replay()
    torch.cuda.synchronize(dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(replays)]
    for a, b in ev:
        a.record()
        b.record()
    torch.cuda.synchronize(dev)
    for a, b in ev:
        a.record()
        g.replay()
        b.record()
    torch.cuda.synchronize(dev)
    per = sorted(a.elapsed_time(b) * 1e3 / G for a, b in ev)  # us per env step of all T tables
    errs = _native.F_OOB | _native.F_AFTER_TERMINAL | _native.F_RNG_LIMIT | _native.F_FAULT
    bad = sum(int(((ch["eng"].flags & errs) != 0).sum().item()) for ch in chains)
    out = {"tables": T, "chains": C, "tables_per_chain": n, "graph_steps": G, "replays": replays,
           "us_per_env_step": {"min": round(per[0], 3), "median": round(per[len(per) // 2], 3), "max": round(per[-1], 3)},
           "env_steps_per_s": round(T / (per[len(per) // 2] * 1e-6), 1), "error_flags": bad}
    for ch in chains:
        ch["eng"].close()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tables", type=int, default=65536)
    ap.add_argument("--chains", default="1,2,4")
    ap.add_argument("--graph-steps", type=int, default=128)
    ap.add_argument("--replays", type=int, default=8)
    ap.add_argument("--warm", type=int, default=2)
    ap.add_argument("--rounds", type=int, default=2, help="alternate the chain counts this many times")
    ap.add_argument("--eager", action="store_true", help="eager launches on C streams instead of one hipGraph")
    ap.add_argument("--offsets", default="0", help="eager: start offsets of chain c (c x this many GPU cycles), comma list")
    a = ap.parse_args()
    for r in range(a.rounds):
        for C in [int(x) for x in a.chains.split(",")]:
            for off in ([int(x) for x in a.offsets.split(",")] if a.eager and C > 1 else [0]):
                print(json.dumps(dict(run(a.tables, C, a.graph_steps, a.replays, a.warm, eager=a.eager,
                                          offset_cycles=off), round=r)), flush=True)


if __name__ == "__main__":
    main()
