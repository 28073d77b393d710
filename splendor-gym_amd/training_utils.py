"""The reference's training_utils.py (training_utils.py:1-282) for the GPU-backed package: every
name ppo_splendor.py:17-24 imports, with the reference signatures.

    make_env              :198-234  env construction (SelfPlay / DualStepSelfPlay / DualStepNative wrapper)
    run_evaluation_suite  :237-260  greedy model vs random, greedy_v1, basic_priority and itself
    frozen_policy_from    :263-276  masked-argmax callable over a frozen ActorCritic copy
    linear_lr_schedule    :279-281
    CheckpointManager     :179-195  latest + timestamped state_dict files
    TrainingLogger        :49-176   TensorBoard scalars, history, summary plot

TensorBoard and matplotlib are optional here (neither is installed in this image): without them
TrainingLogger records the history and writes no event files / PNGs (a one-line notice instead),
everything else behaves as the reference.  The env-step hot path is not in this module.
"""
import os
import sys
from dataclasses import dataclass, field
from datetime import datetime
from typing import Dict, List

import numpy as np
import torch
import torch.nn as nn

from splendor_gym.envs import SplendorEnv
from splendor_gym.scripts.eval_suite import (basic_priority_opponent, eval_vs_opponent, greedy_opponent_v1,  # noqa: F401
                                             make_selfplay_env_with, model_greedy_policy_from)
from splendor_gym.wrappers.selfplay import SelfPlayWrapper, random_opponent

__all__ = ["TrainingHistory", "TrainingLogger", "CheckpointManager", "make_env", "run_evaluation_suite",
           "frozen_policy_from", "linear_lr_schedule", "random_opponent"]


def _summary_writer(log_dir):
    try:
        from torch.utils.tensorboard import SummaryWriter
    except ImportError:  # tensorboard absent
        print("[training_utils] tensorboard is not installed: --track logs nothing", file=sys.stderr)
        return None
    return SummaryWriter(log_dir)


def _pyplot():
    try:
        import matplotlib
        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
        return plt
    except ImportError:
        return None


@dataclass
class TrainingHistory:
    steps: List[int] = field(default_factory=list)
    wr_rand: List[float] = field(default_factory=list)
    wr_greedy1: List[float] = field(default_factory=list)
    wr_basic: List[float] = field(default_factory=list)
    wr_self: List[float] = field(default_factory=list)
    turns_rand: List[float] = field(default_factory=list)
    turns_greedy1: List[float] = field(default_factory=list)
    turns_basic: List[float] = field(default_factory=list)
    turns_self: List[float] = field(default_factory=list)
    lr: List[float] = field(default_factory=list)
    pol_loss: List[float] = field(default_factory=list)
    val_loss: List[float] = field(default_factory=list)
    entropy: List[float] = field(default_factory=list)


# evaluation-result keys -> (win-rate list, turns list) of TrainingHistory
_HIST = {"random": ("wr_rand", "turns_rand"), "greedy_v1": ("wr_greedy1", "turns_greedy1"),
         "basic": ("wr_basic", "turns_basic"), "self_play": ("wr_self", "turns_self")}


class TrainingLogger:
    """Scalars to TensorBoard when `track` (and TensorBoard is installed), an in-memory history,
    and a 2x2 summary figure (win rates, turns, losses, learning rate) when matplotlib is."""

    def __init__(self, log_dir: str, track: bool = False):
        self.log_dir = log_dir
        self.writer = _summary_writer(log_dir) if track else None
        self.history = TrainingHistory()
        self.run_start_ts = datetime.now().strftime("%Y%m%d_%H%M%S")

    def log_training_metrics(self, global_step: int, lr: float, policy_loss: float, value_loss: float,
                             entropy: float, approx_kl: float):
        if self.writer is None:
            return
        for tag, v in (("charts/learning_rate", lr), ("losses/policy_loss", policy_loss),
                       ("losses/value_loss", value_loss), ("losses/entropy", entropy), ("losses/approx_kl", approx_kl)):
            self.writer.add_scalar(tag, v, global_step)

    def log_evaluation_results(self, results: Dict[str, Dict], global_step: int):
        if self.writer is None:
            return
        for name, res in results.items():
            key = name.replace("_", "")
            self.writer.add_scalar(f"eval/win_rate_{key}", res["win_rate"], global_step)
            self.writer.add_scalar(f"eval/win_rate_{key}_ci95", res["win_rate_ci95"], global_step)
            self.writer.add_scalar(f"eval/avg_turns_{key}", res["avg_turns"], global_step)
        if "random" in results:
            r = results["random"]
            self.writer.add_scalar("eval/draw_rate_random", r["draws"] / max(1, r["n"]), global_step)
        if "greedy_v1" in results:
            self.writer.add_scalar("eval/avg_prestige", results["greedy_v1"]["avg_prestige"], global_step)

    def update_history(self, global_step: int, results: Dict[str, Dict], lr: float, policy_loss: float,
                       value_loss: float, entropy: float):
        h = self.history
        h.steps.append(global_step)
        for name, (wr, turns) in _HIST.items():
            getattr(h, wr).append(results.get(name, {}).get("win_rate", 0))
            getattr(h, turns).append(results.get(name, {}).get("avg_turns", 0))
        h.lr.append(lr)
        h.pol_loss.append(policy_loss)
        h.val_loss.append(value_loss)
        h.entropy.append(entropy)

    def create_summary_plot(self, global_step: int) -> bool:
        """summary_<run ts>.png and summary.png in log_dir; False (nothing written) without matplotlib."""
        plt = _pyplot()
        if plt is None:
            return False
        try:
            h = self.history
            fig, ax = plt.subplots(2, 2, figsize=(10, 7))
            labels = (("random", "random"), ("greedy_v1", "greedy_v1"), ("basic", "basic_priority"), ("self_play", "self_play"))
            for key, label in labels:
                ax[0, 0].plot(h.steps, getattr(h, _HIST[key][0]), label=label)
                ax[0, 1].plot(h.steps, getattr(h, _HIST[key][1]), label=label)
            ax[0, 0].set_ylim(0, 1.0)
            ax[0, 0].set(title="Win Rates", xlabel="steps", ylabel="win rate")
            ax[0, 1].set(title="Avg Turns", xlabel="steps", ylabel="turns")
            if len(h.turns_rand) > 1:
                recent = float(np.mean(h.turns_rand[-5:]))
                ax[0, 1].axhline(y=recent, color="red", linestyle="--", alpha=0.5, label=f"Recent avg: {recent:.1f}")
            x = list(range(len(h.pol_loss)))
            for series, label in ((h.pol_loss, "policy"), (h.val_loss, "value"), (h.entropy, "entropy")):
                ax[1, 0].plot(x, series, label=label)
            ax[1, 0].set(title="Losses / Entropy", xlabel="updates")
            ax[1, 1].plot(list(range(len(h.lr))), h.lr, label="lr")
            ax[1, 1].set(title="Learning Rate", xlabel="updates")
            for a in (ax[0, 0], ax[0, 1], ax[1, 0]):
                a.legend()
            fig.suptitle(f"Summary @ {datetime.now().strftime('%Y-%m-%d %H:%M:%S')}")
            fig.tight_layout(rect=[0, 0.03, 1, 0.95])
            if self.writer is not None:
                self.writer.add_figure("eval/summary", fig, global_step)
            fig.savefig(os.path.join(self.log_dir, f"summary_{self.run_start_ts}.png"))
            fig.savefig(os.path.join(self.log_dir, "summary.png"))
            plt.close(fig)
            return True
        except Exception as e:  # the reference swallows plotting errors too
            print(f"[warn] plotting failed: {e}")
            return False


class CheckpointManager:
    def __init__(self, log_dir: str, run_start_ts: str):
        self.log_dir = log_dir
        self.run_start_ts = run_start_ts

    def save_checkpoint(self, model: nn.Module, suffix: str = ""):
        """state_dict to <log_dir>/ppo_splendor_latest<suffix>.pt and checkpoints/ppo_splendor_<ts><suffix>.pt."""
        latest = os.path.join(self.log_dir, f"ppo_splendor_latest{suffix}.pt")
        ts_dir = os.path.join(self.log_dir, "checkpoints")
        os.makedirs(ts_dir, exist_ok=True)
        stamped = os.path.join(ts_dir, f"ppo_splendor_{self.run_start_ts}{suffix}.pt")
        for path in (latest, stamped):
            torch.save(model.state_dict(), path)
        return latest, stamped


def make_env(seed: int, opponent_policy=None, opponent_supplier=None, random_starts: bool = False,
             use_dual_step: bool = False, use_dual_player: bool = True):
    """Thunk building one 2-player SplendorEnv behind a self-play wrapper, reset with `seed`:
    DualStepNativeWrapper when use_dual_player (default), else DualStepSelfPlayWrapper when
    use_dual_step, else SelfPlayWrapper.  The opponent defaults to random_opponent."""
    if opponent_policy is None and opponent_supplier is None:
        opponent_policy = random_opponent

    def thunk():
        env = SplendorEnv(num_players=2)
        if use_dual_player:
            from splendor_gym.wrappers.dual_step_native import DualStepNativeWrapper as W
        elif use_dual_step:
            from splendor_gym.wrappers.dual_step_selfplay import DualStepSelfPlayWrapper as W
        else:
            W = SelfPlayWrapper
        env = W(env, opponent_policy=opponent_policy or random_opponent, opponent_supplier=opponent_supplier,
                random_starts=random_starts)
        env.reset(seed=seed)
        return env

    return thunk


def run_evaluation_suite(agent: nn.Module, device: torch.device, rng: np.random.RandomState, n_games: int,
                         update_seed: int = 0) -> Dict[str, Dict]:
    """Greedy agent vs random, greedy_v1, basic_priority and a greedy copy of itself; each env
    factory reseeds from `rng`, each evaluation from update_seed + i (training_utils.py:237-260)."""
    policy = model_greedy_policy_from(agent, device=device)
    opponents = [("random", random_opponent), ("greedy_v1", greedy_opponent_v1), ("basic", basic_priority_opponent),
                 ("self_play", model_greedy_policy_from(agent, device=device))]
    results = {}
    for i, (name, opp) in enumerate(opponents):
        def env_fn(opp=opp):
            return make_selfplay_env_with(opp, int(rng.randint(1e9)))()
        results[name] = eval_vs_opponent(env_fn, policy, n_games=n_games, seed=update_seed + i)
    return results


def frozen_policy_from(state_dict: dict, actor_critic_class, obs_dim: int, act_dim: int, device: torch.device):
    """Masked-argmax policy of a frozen `actor_critic_class(obs_dim, act_dim)` loaded from state_dict."""
    frozen = actor_critic_class(obs_dim, act_dim).to(device)
    frozen.load_state_dict(state_dict)
    frozen.eval()

    @torch.no_grad()
    def _policy(obs, info):
        x = torch.tensor(obs, dtype=torch.float32, device=device).unsqueeze(0)
        m = torch.tensor(info["action_mask"], dtype=torch.float32, device=device).unsqueeze(0)
        return int(torch.argmax(frozen.actor(x).masked_fill(m < 0.5, float("-inf")), dim=-1).item())
    _policy.frozen_model = frozen  # batched self-play reads the weights (splendor_gym.selfplay)
    return _policy


def linear_lr_schedule(initial_lr: float, progress: float) -> float:
    return initial_lr * progress
