"""DualStepNativeWrapper: dual_step(a) plays the agent's move and the opponent's reply and
returns both players' data.  Drop-in for reference splendor_gym/wrappers/dual_step_native.py:6-223
(the wrapper ppo_splendor.py drives through envs.envs[i].dual_step)."""
from typing import Any, Callable, Dict, Optional, Tuple

import numpy as np

from .._gym_compat import Wrapper
from ._common import episode_opponent, final_reward, play_opening, random_opponent  # noqa: F401


class DualStepNativeWrapper(Wrapper):
    def __init__(self, env, opponent_policy: Callable, random_starts: bool = True,
                 opponent_supplier: Optional[Callable] = None):
        super().__init__(env)
        self.opponent_policy = opponent_policy
        self.random_starts = random_starts
        self.opponent_supplier = opponent_supplier
        self._opp_policy = opponent_policy
        self.turn_count = 0
        self.total_agent_steps = 0
        self.total_opponent_steps = 0

    def _to_play(self):
        """Player to move, or None before reset.  The reference reads env.state.to_play
        (dual_step_native.py:94-97, 130); the GPU env answers from its last observation (or from
        an outstanding write-through view) instead of downloading the table, so a dual step costs
        two env steps and no state downloads."""
        cached = getattr(self.env, "cached_to_play", None)
        if cached is not None:
            return cached()
        state = getattr(self.env, "state", None)
        return None if state is None else state.to_play

    def _count_opponent(self):
        self.total_opponent_steps += 1

    def reset(self, **kwargs):
        self._opp_policy = episode_opponent(self)
        obs, info = self.env.reset(**kwargs)
        self.turn_count = self.total_agent_steps = self.total_opponent_steps = 0
        return play_opening(self, obs, info, self._count_opponent)

    def step(self, action: int):
        """Agent-perspective view of dual_step (truncation is never used)."""
        agent_obs, agent_reward, _, _, done, info = self.dual_step(action)
        return agent_obs, agent_reward, done, False, info

    def dual_step(self, agent_action: int) -> Tuple[np.ndarray, float, np.ndarray, float, bool, Dict[str, Any]]:
        """(agent_obs, agent_reward, opponent_obs, opponent_reward, done, info) after the agent's
        move and, unless that ended the game, the opponent's reply (dual_step_native.py:90-193).
        Both observation slots hold the same array: the encoding is from the side to play."""
        if self._to_play() is None:
            raise RuntimeError("Cannot call dual_step() before reset()")
        if self._to_play() != 0:
            raise ValueError("dual_step() requires agent (player 0) to move first")
        self.turn_count += 1
        self.total_agent_steps += 1
        obs_a, rew_a, done_a, trunc_a, info_a = self.env.step(agent_action)
        info = {"turn_count": self.turn_count, "agent_action": agent_action,
                "total_agent_steps": self.total_agent_steps, "total_opponent_steps": self.total_opponent_steps,
                "phase": "agent_only"}
        info.update(info_a)
        if done_a or trunc_a:
            opp_reward = final_reward(info_a, 1)
            info.update({"opponent_action": None, "opponent_reward": opp_reward, "turn_complete": True,
                         "game_ended_on": "agent_move"})
            return obs_a, rew_a, obs_a, opp_reward, True, info
        to_play = self._to_play()
        if to_play != 1:
            raise ValueError(f"Expected opponent (player 1) to move after agent, got to_play={to_play}")
        opp_action = self._opp_policy(obs_a, info_a)
        self.total_opponent_steps += 1
        obs_o, rew_o, done_o, trunc_o, info_o = self.env.step(opp_action)
        ended = done_o or trunc_o
        info.update(info_o)
        info.update({"opponent_action": opp_action, "opponent_reward": rew_o,
                     "total_opponent_steps": self.total_opponent_steps, "phase": "complete_turn",
                     "turn_complete": True, "game_ended_on": "opponent_move" if ended else None})
        return obs_o, (final_reward(info_o, 0) if ended else 0.0), obs_o, rew_o, done_o, info

    def get_wrapper_stats(self) -> Dict[str, Any]:
        return {"turn_count": self.turn_count, "total_agent_steps": self.total_agent_steps,
                "total_opponent_steps": self.total_opponent_steps,
                "avg_opponent_steps_per_turn": self.total_opponent_steps / max(1, self.turn_count),
                "wrapper_type": "DualStepNativeWrapper"}
