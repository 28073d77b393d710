"""The reference evaluation module (splendor_gym/scripts/eval_suite.py:1-253), same names and
signatures, over the GPU-backed env: what ppo_splendor.py:11-16 and training_utils.py:22-28 import.

Per-env callables `(obs int32[297], info{action_mask int8[45]}) -> action`:
    random_opponent (wrappers/selfplay.py:66-73), greedy_opponent_v1 (:10-30),
    basic_priority_opponent (:33-77), greedy_opponent_v2_factory (:80-128),
    model_greedy_policy_from (:131-141)
Per-game evaluation loops with the reference's seeding and statistics:
    make_selfplay_env / make_selfplay_env_with (:144-159), eval_vs_opponent (:162-208),
    eval_vs_checkpoint_pool (:211-253)

The loops play one SplendorEnv (one device table) at a time, exactly like the reference.  For
batched evaluation (all games of a run in one launch per ply) use
splendor_gym.evaluation.eval_vs_opponent — same statistics, pinned to the same fixtures.
"""
from typing import Any, Callable, Dict, List

import numpy as np
import torch

from ..engine.encode import OBSERVATION_DIM, TOTAL_ACTIONS, TAKE3_COMBOS  # noqa: F401
from ..envs import SplendorEnv
from ..opponents import basic_priority_opponent, greedy_opponent_v1  # noqa: F401
from ..wrappers.selfplay import SelfPlayWrapper, random_opponent  # noqa: F401

__all__ = ["random_opponent", "greedy_opponent_v1", "basic_priority_opponent", "greedy_opponent_v2_factory",
           "model_greedy_policy_from", "make_selfplay_env", "make_selfplay_env_with", "eval_vs_opponent",
           "eval_vs_checkpoint_pool"]


def greedy_opponent_v2_factory(env_ref=None) -> Callable:
    """Buys first (visible, then reserved, in id order); else the take-2 / take-3 of the scarcest
    bank colours (bank read from env_ref.state, uniform without it); else the highest-index reserve."""
    def policy(obs, info):
        legal = np.flatnonzero(info["action_mask"])
        if len(legal) == 0:
            return 0
        buys = [a for a in legal if 15 <= a <= 26] + [a for a in legal if 42 <= a <= 44]
        if buys:
            return int(buys[0])
        bank = list(env_ref.state.bank[:5]) if getattr(env_ref, "state", None) is not None else [1] * 5
        take2 = [a for a in legal if 10 <= a <= 14]
        if take2:
            return int(min(take2, key=lambda a: bank[a - 10]))
        take3 = [a for a in legal if a <= 9]
        if take3:
            return int(min(take3, key=lambda a: sum(bank[c] for c in TAKE3_COMBOS[a])))
        res = [a for a in legal if 27 <= a <= 41]
        return int(max(res)) if res else int(legal[0])
    return policy


def model_greedy_policy_from(model: torch.nn.Module, device: str = "cpu") -> Callable[[np.ndarray, Dict[str, Any]], int]:
    """Masked argmax of model.actor(obs) for one env (batch of one, fp32)."""
    model.eval()

    @torch.no_grad()
    def _policy(obs, info):
        x = torch.tensor(obs, dtype=torch.float32, device=device).unsqueeze(0)
        m = torch.tensor(info["action_mask"], dtype=torch.float32, device=device).unsqueeze(0)
        logits = model.actor(x).masked_fill(m < 0.5, float("-inf"))
        return int(torch.argmax(logits, dim=-1).item())
    return _policy


def make_selfplay_env_with(opponent_policy: Callable, seed: int):
    """Thunk: 2-player SplendorEnv behind SelfPlayWrapper(opponent_policy), reset with `seed`."""
    def thunk():
        env = SelfPlayWrapper(SplendorEnv(num_players=2), opponent_policy=opponent_policy)
        env.reset(seed=seed)
        return env
    return thunk


def make_selfplay_env(seed: int):
    return make_selfplay_env_with(random_opponent, seed)


def eval_vs_opponent(make_env: Callable[[], Any], model_policy: Callable, n_games: int = 400,
                     seed: int = 0) -> Dict[str, Any]:
    """`n_games` games of model_policy (player 0) against the env's opponent.  Game g resets with
    np.random.RandomState(seed).randint(1e9) draw g; the result is the sign of the final reward
    the wrapper returns; avg_turns / avg_prestige read the final state (prestige of the player
    who moved last); illegal_action_rate counts choices outside the mask."""
    rng = np.random.RandomState(seed)
    wins = losses = draws = 0
    turns: List[int] = []
    prestige: List[int] = []
    illegal = checks = 0
    for _ in range(n_games):
        env = make_env()
        obs, info = env.reset(seed=int(rng.randint(1e9)))
        while True:
            checks += 1
            a = model_policy(obs, info)
            if info["action_mask"][a] == 0:
                illegal += 1
            obs, r, term, trunc, info = env.step(a)
            if term or trunc:
                if r > 0:
                    wins += 1
                elif r < 0:
                    losses += 1
                else:
                    draws += 1
                break
        s = env.env.state
        turns.append(s.turn_count)
        prestige.append(s.players[(s.to_play - 1) % s.num_players].prestige)
        env.close()
    p = wins / max(1, n_games)
    return {"n": n_games, "wins": wins, "losses": losses, "draws": draws, "win_rate": p,
            "win_rate_ci95": 1.96 * np.sqrt(p * (1 - p) / max(1, n_games)),
            "avg_turns": float(np.mean(turns)) if turns else 0.0,
            "avg_prestige": float(np.mean(prestige)) if prestige else 0.0,
            "illegal_action_rate": float(illegal / max(1, checks))}


def eval_vs_checkpoint_pool(checkpoint_paths: List[str], model_policy: Callable, n_games: int = 400,
                            seed: int = 0) -> Dict[str, Any]:
    """The reference splits n_games over the paths but plays each share against a uniformly random
    opponent (it never loads the checkpoints, eval_suite.py:221-229); kept as is."""
    empty = {"n": 0, "wins": 0, "losses": 0, "draws": 0, "win_rate": 0.0, "win_rate_ci95": 0.0, "avg_turns": 0.0,
             "avg_prestige": 0.0, "illegal_action_rate": 0.0}
    if not checkpoint_paths:
        return empty
    rng = np.random.RandomState(seed)
    per = max(1, n_games // len(checkpoint_paths))
    res_all = []
    for _ in checkpoint_paths:
        env_fn = make_selfplay_env_with(random_opponent, int(rng.randint(1e9)))
        res_all.append(eval_vs_opponent(env_fn, model_policy, n_games=per, seed=int(rng.randint(1e9))))
    n = max(1, sum(r["n"] for r in res_all))
    wins = sum(r["wins"] for r in res_all)
    p = wins / n
    return {"n": n, "wins": wins, "losses": sum(r["losses"] for r in res_all), "draws": sum(r["draws"] for r in res_all),
            "win_rate": p, "win_rate_ci95": 1.96 * np.sqrt(p * (1 - p) / n),
            "avg_turns": float(np.mean([r["avg_turns"] for r in res_all])),
            "avg_prestige": float(np.mean([r["avg_prestige"] for r in res_all])),
            "illegal_action_rate": float(sum(r["illegal_action_rate"] * r["n"] for r in res_all) / n)}
