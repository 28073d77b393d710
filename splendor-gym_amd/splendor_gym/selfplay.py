"""Batched two-player self-play: DualStepNativeWrapper.dual_step for N tables per launch.

`DualStepVectorEnv.dual_step(actions)` plays, on every table, the agent's move (player 0) and the
opponent's reply, with the results of reference wrappers/dual_step_native.py:90-193 per table, and
re-deals finished tables the way the PPO loop does after `done` (ppo_splendor.py:246-256).  It is
the device form of `envs.envs[i].dual_step(a)` in a Python loop: two spl_step launches (agent move;
opponent move) with the opponent's actions computed in between on the device, by

  * a device policy fused into the agent-move kernel: "random" (wrappers/selfplay.py:66-73),
    "greedy_v1" / "basic_priority" (scripts/eval_suite.py:9-78; random choices are Philox draws),
  * or any batched callable (obs int32 [N,297], mask int8 [N,45]) -> actions [N], e.g.
    splendor_gym.policy.greedy_opponent_from(actor) for self-play against a network
    (eval_suite.py:131-141 model_greedy_policy_from).

Per table (reference semantics):
  * the agent's move ends the game (only the no-legal-move draw can: terminal needs to_play == 0):
    agent_reward = its step reward, opponent_reward = final_rewards[1] (0 without them),
    no opponent move;
  * otherwise the opponent moves: agent_reward = final_rewards[0] if that ended the game else 0,
    opponent_reward = the opponent's step reward;
  * an illegal or out-of-range agent action (the reference raises ValueError) leaves the table
    unchanged with the agent still to play: the opponent does not move, rewards 0 and -0.01 is
    reported in info["agent_step_reward"]; info["illegal_action"] marks it.
Finished tables are re-dealt in the same call (the next episode of the table's engine-seed
stream); `agent_obs` / info["action_mask"] are then the new episode's, info["final_observation"]
holds the observation that ended the game, and `opp_obs` is the reference's opponent_obs (the
post-turn observation, i.e. the final one on finished tables) when requested.
"""
import torch

from . import _native
from .device import Engine

_DEVICE_POLICIES = {"random": _native.POLICY_UNIFORM, "greedy_v1": _native.POLICY_GREEDY_V1,
                    "basic_priority": _native.POLICY_BASIC_PRIORITY}


class DualStepVectorEnv:
    def __init__(self, num_envs, device=None, opponent="random", policy_seed=0, refill_period=None, table0=0,
                 opponent_obs=True):
        if isinstance(opponent, str) and opponent not in _DEVICE_POLICIES:
            raise ValueError(f"unknown device opponent {opponent!r}; choose {sorted(_DEVICE_POLICIES)} or a callable")
        self.eng = Engine(num_envs, 2, device=device, refill_period=refill_period, table0=table0)
        self.num_envs, self.device = num_envs, self.eng.device
        self.opponent = opponent
        self.policy_seed = int(policy_seed)
        self.want_opp_obs = opponent_obs
        t = torch
        n, dev = num_envs, self.device
        self.opp_actions = t.zeros(n, dtype=t.int32, device=dev)
        self.agent_reward = t.zeros(n, dtype=t.float32, device=dev)
        self.opp_reward = t.zeros(n, dtype=t.float32, device=dev)
        self._ply = 0

    # ------------------------------------------------------------------------------------
    def reset(self, seed=None, seeds=None):
        """Deal every table (env i seeded with seed + i, or seeds[i]; neither: continue each
        table's stream).  A fresh deal has player 0 to play, so the reference's opening loop never
        moves the opponent here (dual_step_native.py:60-77)."""
        if seeds is None and seed is not None:
            seeds = range(int(seed), int(seed) + self.num_envs)
        obs, mask = self.eng.reset(seeds=seeds)
        return obs, {"action_mask": mask, "to_play": obs[:, 294]}

    @staticmethod
    def _final_reward(player, winner, flags):
        """final_rewards[player] (envs/splendor_env.py:92-115): ±1, or 0 / -0.1 (turn limit) when
        there is no winner; 0 for the no-legal-move draw, which reports none."""
        tl = (flags & _native.F_TURN_LIMIT) != 0
        no_winner = torch.where(tl, torch.full_like(winner, -0.1, dtype=torch.float32),
                                torch.zeros_like(winner, dtype=torch.float32))
        return torch.where(winner < 0, no_winner,
                           torch.where(winner == player, 1.0, -1.0).to(torch.float32))

    def dual_step(self, actions):
        e = self.eng
        device_opp = isinstance(self.opponent, str)
        self._ply += 1
        # phase A: the agent's move (no reset); a device opponent's reply is drawn in the same kernel
        e.step(actions, autoreset=False, final_obs=False,
               next_actions=self.opp_actions if device_opp else None,
               policy=_DEVICE_POLICIES[self.opponent] if device_opp else 0,
               policy_seed=self.policy_seed, ply=self._ply)
        # keep phase A's small outputs: the opponent move overwrites the engine's buffers
        ra, ta, fa, wa = e.reward.clone(), e.terminated.clone(), e.flags.clone(), e.winner.clone()
        passed = (ta == 0) & ((fa & (_native.F_ILLEGAL | _native.F_OOB)) == 0)  # player 1 is to play
        if device_opp:
            opp = self.opp_actions
        else:
            opp = torch.as_tensor(self.opponent(e.obs, e.mask), device=self.device).to(torch.int32)
        opp = torch.where(passed, opp, torch.full_like(opp, -1))  # -1: out of range, no move
        # phase B: the opponent's move; autoreset 2 also re-deals tables that ended on the agent's move
        e.step(opp, autoreset=2, final_obs=True)
        tb, fb, wb, rb = e.terminated, e.flags, e.winner, e.reward
        ended_a, ended_b = ta != 0, tb != 0
        done = ended_a | ended_b
        torch.where(ended_a, ra, torch.where(ended_b, self._final_reward(0, wb, fb), torch.zeros_like(rb)),
                    out=self.agent_reward)
        torch.where(ended_a, self._final_reward(1, wa, fa), torch.where(passed, rb, torch.zeros_like(rb)),
                    out=self.opp_reward)
        agent_obs = e.obs
        opp_obs = torch.where(done[:, None], e.final_obs, e.obs) if self.want_opp_obs else None
        info = {"action_mask": e.mask, "to_play": e.obs[:, 294], "final_observation": e.final_obs,
                "opponent_action": torch.where(passed, opp, torch.full_like(opp, -1)),
                "game_ended_on": torch.where(ended_a, 1, torch.where(ended_b, 2, 0)).to(torch.int8),
                "illegal_action": (fa & _native.F_ILLEGAL) != 0, "agent_step_reward": ra,
                "draw": ((fa | fb) & _native.F_DRAW) != 0, "turn_limit": ((fa | fb) & _native.F_TURN_LIMIT) != 0}
        return agent_obs, self.agent_reward, opp_obs, self.opp_reward, done, info

    def close(self):
        self.eng.close()
