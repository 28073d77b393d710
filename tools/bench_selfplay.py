"""BASELINE config 5: 2-player self-play with the PPO actor on device (ppo_splendor.py:227-269).

    python tools/bench_selfplay.py [--tables 65536] [--iters 64] [--warmup 16] [--bf16]
    torchrun --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 tools/bench_selfplay.py ...

One iteration = the PPO rollout step for every table: the agent's ActorCritic forward
(get_action_and_value: actor + critic + masked categorical sample) on the current observations,
then DualStepVectorEnv.dual_step (agent move, the opponent's greedy reply from a frozen
ActorCritic — eval_suite.py:131-141 — and the reset of finished tables).  A dual step is 2
env-steps.  Weights are random-initialised (no checkpoint travels); compute is
fp32 like the reference unless --bf16.  Prints one JSON line on rank 0 (weak scaling: tables per
GPU fixed, max-over-ranks time), plus the env-only share measured with the actor forward removed.
"""
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
    ap.add_argument("--iters", type=int, default=64)
    ap.add_argument("--warmup", type=int, default=16)
    ap.add_argument("--bf16", action="store_true",
                    help="opt-in reduced precision: the fused kernel's bf16 MFMA image, or the torch actor under bf16 "
                         "autocast (default fp32, the reference's precision)")
    ap.add_argument("--actor", choices=["fused", "torch"], default="fused",
                    help="fused: spl_policy_act (fp32-accurate split-bf16 kernel, bf16 with --bf16) for agent and opponent; "
                         "torch: the nn.Module")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--graph-steps", type=int, default=4, help="dual steps captured per hipGraph (bench.py: 4)")
    ap.add_argument("--opponent", choices=["pool", "frozen"], default="pool",
                    help="pool: the reference's opponent_supplier (current policy p=0.25, else one of 12 frozen "
                         "snapshots, drawn per episode; fused fp32 grouped kernel); frozen: one frozen greedy actor")
    ap.add_argument("--pool-size", type=int, default=12)
    ap.add_argument("--weights", choices=["trained", "random"], default="trained",
                    help="trained: the reference's runs/ppo_splendor/ppo_splendor_latest.pt (committed as "
                         "tests/golden/ppo_splendor_latest.safetensors) for agent, opponent and pool snapshots; "
                         "random: random-init networks")
    args = ap.parse_args()

    import torch
    from splendor_gym.parallel import barrier, init_distributed, local_device, max_over_ranks
    from splendor_gym.fused_policy import FusedActorCritic, OpponentPool
    from splendor_gym.policy import ActorCritic, greedy_opponent_from
    from splendor_gym.selfplay import DualStepVectorEnv

    rank, world, local = init_distributed()
    dev = local_device(local)
    torch.cuda.set_device(dev)
    torch.manual_seed(1234 + rank)
    N = args.tables
    ckpt = os.path.join(REPO, "tests", "golden", "ppo_splendor_latest.safetensors")

    def net():
        m = ActorCritic().to(dev).eval()
        if args.weights == "trained":
            from safetensors.torch import load_file
            m.load_state_dict(load_file(ckpt, device=str(dev)))
        return m

    agent = net()
    opp_model = net()
    fused = args.actor == "fused"
    if fused:
        prec = "bf16" if args.bf16 else "fp32"
        agent_k = FusedActorCritic(agent, precision=prec)
        if args.opponent == "pool":
            if args.bf16:
                raise SystemExit("--opponent pool is fp32 (the grouped kernel); use --opponent frozen with --bf16")
            opponent = OpponentPool(agent, pool_size=args.pool_size, p_current=0.25, seed=99)
            for _ in range(args.pool_size):  # one snapshot image per slot (the one checkpoint, or random init)
                opponent.add_snapshot(net())
        else:
            opponent = FusedActorCritic(opp_model, with_critic=False, precision=prec).opponent()
    else:
        opponent = greedy_opponent_from(opp_model)
    ply_t = torch.zeros(1, dtype=torch.int64, device=dev)  # advanced by each dual step's last launch
    env = DualStepVectorEnv(N, device=dev, opponent=opponent, table0=rank * N, opponent_obs=False,
                            step_counter=ply_t if fused else None, agent_obs_u8=fused and not args.bf16)
    obs, info = env.reset(seed=rank * N)
    mask = info["action_mask"]
    amp = torch.autocast("cuda", dtype=torch.bfloat16) if (args.bf16 and not fused) else torch.autocast("cuda", enabled=False)

    def iteration(with_actor=True):
        with torch.no_grad(), amp:
            if with_actor and fused:
                a, logprob, entropy, value = agent_k.act(obs if env.agent_obs_u8 is None else env.agent_obs_u8, mask,
                                                         seed=1234, table0=rank * N, ply_base=ply_t)
            elif with_actor:
                action, logprob, _, value = agent.get_action_and_value(obs.float(), mask.float())
                a = action.to(torch.int32)
            else:
                a = env.eng.sample_uniform(mask=mask, out=env.opp_actions.clone(), seed=7, ply=0)
            return env.dual_step(a)

    for _ in range(args.warmup):
        iteration()
    graph = None
    if not args.no_graph:
        try:
            torch.cuda.synchronize(dev)
            s = torch.cuda.Stream(device=dev)
            s.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(s):
                for _ in range(2):
                    iteration()
            torch.cuda.current_stream(dev).wait_stream(s)
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                for _ in range(args.graph_steps):
                    iteration()
        except Exception as exc:  # capture unsupported: eager
            print(f"graph capture failed ({exc}); timing eager iterations", file=sys.stderr)
            graph = None

    def timed(fn, iters):
        barrier(dev)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(iters):
            fn()
        torch.cuda.synchronize(dev)
        barrier(dev)
        return max_over_ranks(time.perf_counter() - t0, device=dev)

    if graph is not None:  # whole graphs of graph_steps dual steps
        args.iters = max(args.graph_steps, args.iters - args.iters % args.graph_steps)
    full = (timed(graph.replay, args.iters // args.graph_steps) if graph is not None else timed(iteration, args.iters))
    env_only = timed(lambda: iteration(with_actor=False), args.iters)
    if rank == 0:
        steps = 2 * N * world * args.iters
        print(json.dumps({
            "metric": f"env-steps/sec (whole node), 2p self-play with on-device ActorCritic actor, {N} tables/GPU",
            "value": round(steps / full, 1), "unit": "env-steps/s", "n_gpus": world, "iters": args.iters,
            "ms_per_dual_step": round(full / args.iters * 1e3, 4), "higher_is_better": True, "scaling": "weak",
            "dtype": "bf16" if args.bf16 else "fp32 (three bf16 planes per operand, fp32 accumulation)", "data": ("synthetic: seeded deals; ActorCritic weights from the reference checkpoint "
                     "runs/ppo_splendor/ppo_splendor_latest.pt (agent, opponent, every pool snapshot)"
                     if args.weights == "trained" else "synthetic: seeded deals, random-init ActorCritic"),
            "config": {"workload": "PPO rollout step: ActorCritic.get_action_and_value + DualStepVectorEnv.dual_step "
                                   + ("(opponent pool: current policy p=0.25 else one of "
                                      f"{args.pool_size} frozen snapshots per episode, greedy; reset after done)"
                                      if fused and args.opponent == "pool" else
                                      "(greedy frozen-ActorCritic opponent, reset after done)"),
                       "weights": args.weights, "tables_per_gpu": N, "players": 2, "launch": "hipGraph replay" if graph is not None else "eager",
                       "actor": (f"spl_policy_act (fused, {'bf16 MFMA' if args.bf16 else 'fp32-accurate split-bf16 MFMA'})" if fused
                                 else "torch nn.Module" + (" (bf16 autocast)" if args.bf16 else ""))},
            "env_only": {"value": round(steps / env_only, 1), "ms_per_dual_step": round(env_only / args.iters * 1e3, 4),
                         "note": "same loop with the agent's forward replaced by device uniform sampling (eager)"},
        }))
    env.close()


if __name__ == "__main__":
    main()
