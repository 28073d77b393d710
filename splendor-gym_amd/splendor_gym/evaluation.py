"""Batched evaluation against scripted or network opponents (reference scripts/eval_suite.py).

`eval_vs_opponent` plays `n_games` games at once, one table per game, with the reference's
per-game seeds (np.random.RandomState(seed).randint(1e9) per game) and statistics
(eval_suite.py:162-208), keeping its conventions:
  * the agent is player 0 behind SelfPlayWrapper: when the opponent's move ends the game the
    agent's reward is minus the opponent's step reward (selfplay.py:54-58), so a turn-limit draw
    (-0.1 for the mover) counts as a win, as in the reference;
  * avg_prestige is the prestige of player (to_play - 1) % 2 at the end, i.e. of the opponent;
  * an action outside the legal mask counts toward illegal_action_rate (with no legal move the
    env's draw follows).  The reference then raises from SelfPlayWrapper for a non-empty mask;
    here the table simply stays at the agent's turn.
`agent_policy` is a batched callable (obs int32 [N,297], mask int8 [N,45]) -> actions [N];
`opponent` is a device policy name or a batched callable (see splendor_gym.selfplay).
"""
import numpy as np
import torch

from .selfplay import DualStepVectorEnv

_OPP_PRESTIGE = 30   # obs: the other player's prestige (engine/encode.py:138-142); to_play == 0 at the end
_TURN_COUNT = 293    # obs: turn_count (encode.py:183)


def first_legal_policy(obs, mask):
    """Lowest legal action id (0 with none legal) for every row."""
    return torch.argmax(mask, dim=1).to(torch.int32)


def last_legal_policy(obs, mask):
    """Highest legal action id (0 with none legal) for every row."""
    last = mask.shape[1] - 1 - torch.argmax(torch.flip(mask, dims=[1]), dim=1)
    return torch.where(mask.any(dim=1), last, torch.zeros_like(last)).to(torch.int32)


@torch.no_grad()
def eval_vs_opponent(agent_policy, opponent="greedy_v1", n_games=400, seed=0, device=None, max_turns=1000):
    rng = np.random.RandomState(seed)
    seeds = [int(rng.randint(1e9)) for _ in range(n_games)]
    env = DualStepVectorEnv(n_games, device=device, opponent=opponent, opponent_obs=False)
    try:
        obs, info = env.reset(seeds=seeds)
        dev = env.device
        playing = torch.ones(n_games, dtype=torch.bool, device=dev)
        result = torch.zeros(n_games, dtype=torch.float32, device=dev)
        turns = torch.zeros(n_games, dtype=torch.int32, device=dev)
        prestige = torch.zeros(n_games, dtype=torch.int32, device=dev)
        checks = torch.zeros((), dtype=torch.int64, device=dev)
        illegal = torch.zeros((), dtype=torch.int64, device=dev)
        for _ in range(max_turns):
            mask = info["action_mask"]
            a = torch.as_tensor(agent_policy(obs, mask), device=dev).to(torch.int32)
            legal_a = mask.gather(1, a.clamp(0, mask.shape[1] - 1).long()[:, None])[:, 0] != 0
            checks += playing.sum()
            illegal += (playing & ~legal_a).sum()
            obs, _, _, opp_reward, done, info = env.dual_step(a)
            ended = playing & done
            r = torch.where(info["game_ended_on"] == 1, info["agent_step_reward"], -opp_reward)
            final = info["final_observation"]
            result = torch.where(ended, r, result)
            turns = torch.where(ended, final[:, _TURN_COUNT], turns)
            prestige = torch.where(ended, final[:, _OPP_PRESTIGE], prestige)
            playing &= ~done
            if not bool(playing.any()):
                break
        res = result.cpu().numpy()
        n = n_games
        wins, losses = int((res > 0).sum()), int((res < 0).sum())
        p = wins / max(1, n)
        return {"n": n, "wins": wins, "losses": losses, "draws": n - wins - losses, "win_rate": p,
                "win_rate_ci95": float(1.96 * np.sqrt(p * (1 - p) / max(1, n))),
                "avg_turns": float(turns.double().mean()), "avg_prestige": float(prestige.double().mean()),
                "illegal_action_rate": float(illegal) / max(1, int(checks)),
                "unfinished": int(playing.sum())}
    finally:
        env.close()
