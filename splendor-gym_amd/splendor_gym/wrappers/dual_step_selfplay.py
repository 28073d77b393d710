"""DualStepSelfPlayWrapper: one step() = the agent's move and the opponent's reply, with the
agent's reward taken from final_rewards.  Drop-in for reference
splendor_gym/wrappers/dual_step_selfplay.py:6-180."""
from typing import Any, Callable, Dict, Optional, Tuple

from .._gym_compat import Wrapper
from ._common import episode_opponent, play_opening, random_opponent  # noqa: F401


class DualStepSelfPlayWrapper(Wrapper):
    def __init__(self, env, opponent_policy: Callable, random_starts: bool = True,
                 opponent_supplier: Optional[Callable] = None):
        super().__init__(env)
        self.opponent_policy = opponent_policy
        self.random_starts = random_starts
        self.opponent_supplier = opponent_supplier
        self._opp_policy = opponent_policy
        self.turn_count = 0
        self.total_agent_actions = 0
        self.total_opponent_actions = 0

    def _count_opponent(self):
        self.total_opponent_actions += 1

    def reset(self, **kwargs):
        self._opp_policy = episode_opponent(self)
        obs, info = self.env.reset(**kwargs)
        self.turn_count = self.total_agent_actions = self.total_opponent_actions = 0
        return play_opening(self, obs, info, self._count_opponent)

    def step(self, agent_action: int) -> Tuple[Any, float, bool, bool, Dict]:
        self.turn_count += 1
        self.total_agent_actions += 1
        obs_a, rew_a, done_a, trunc_a, info_a = self.env.step(agent_action)
        info = {"turn_count": self.turn_count, "agent_action": agent_action,
                "total_agent_actions": self.total_agent_actions,
                "total_opponent_actions": self.total_opponent_actions, "phase": "agent_only"}
        info.update(info_a)
        if done_a or trunc_a:  # dual_step_selfplay.py:113-117
            info["game_ended_on"] = "agent_move"
            info["turn_complete"] = True
            return obs_a, rew_a, done_a, trunc_a, info
        if info_a.get("to_play", 0) != 1:  # :153-158
            raise RuntimeError(f"Invalid state after agent move: to_play={info_a.get('to_play', 'unknown')}, "
                               "expected 1 for opponent. Game state may be corrupted.")
        opp_action = self._opp_policy(obs_a, info_a)
        self.total_opponent_actions += 1
        obs_o, rew_o, done_o, trunc_o, info_o = self.env.step(opp_action)
        info.update(info_o)
        info.update({"opponent_action": opp_action, "opponent_reward": rew_o,
                     "total_opponent_actions": self.total_opponent_actions, "phase": "complete_turn",
                     "turn_complete": True})
        if not (done_o or trunc_o):
            return obs_o, 0.0, done_o, trunc_o, info
        info["game_ended_on"] = "opponent_move"  # :138-149: final_rewards[0], else the agent's own reward
        fr = info_o.get("final_rewards")
        agent_reward = fr[0] if fr is not None and 0 in fr else rew_a
        return obs_o, agent_reward, done_o, trunc_o, info

    def get_wrapper_stats(self) -> Dict[str, Any]:
        return {"turn_count": self.turn_count, "total_agent_actions": self.total_agent_actions,
                "total_opponent_actions": self.total_opponent_actions,
                "avg_opponent_actions_per_turn": self.total_opponent_actions / max(1, self.turn_count),
                "wrapper_type": "DualStepSelfPlayWrapper"}
