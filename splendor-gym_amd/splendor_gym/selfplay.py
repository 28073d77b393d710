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
    (eval_suite.py:131-141 model_greedy_policy_from),
  * or an OpponentPool (splendor_gym.fused_policy): the opponent_supplier of ppo_splendor.py:137-143 —
    each table's episode plays the current policy or a frozen snapshot, drawn per table at every
    episode start (info["opponent_index"]: 0 = current, else the snapshot's image slot).

random_starts (dual_step_native.py:61-77): the reference flips a coin only when the opponent is to
play right after reset, and lets it move first on heads — then its loop moves the opponent while it
is to play either way, so heads and tails play the same moves.  A fresh deal always has player 0
to play, so the flip never happens; the flag is accepted for signature parity and changes nothing.

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
import ctypes
from collections.abc import Mapping

import torch

from . import _native
from .device import Engine

_DEVICE_POLICIES = {"random": _native.POLICY_UNIFORM, "greedy_v1": _native.POLICY_GREEDY_V1,
                    "basic_priority": _native.POLICY_BASIC_PRIORITY}


class DualInfo(Mapping):
    """info of a batched dual step.  The boolean views illegal_action / draw / turn_limit are
    derived from the packed info_flags on first access (each is one extra tensor op)."""
    _LAZY = {"illegal_action": _native.DUAL_ILLEGAL, "draw": _native.DUAL_DRAW, "turn_limit": _native.DUAL_TURN_LIMIT}

    def __init__(self, base, info_flags):
        self._d = dict(base)
        self._flags = info_flags

    def __getitem__(self, k):
        if k not in self._d and k in self._LAZY:
            self._d[k] = (self._flags & self._LAZY[k]) != 0
        return self._d[k]

    def __iter__(self):
        return iter(list(self._d) + [k for k in self._LAZY if k not in self._d])

    def __len__(self):
        return len(set(self._d) | set(self._LAZY))


def compact_rows(obs, out):
    """out (uint8 [n, 300]) = the compact rows of int32 observations obs [n, 297] (spl_step_args_t.obs_u8:
    bytes 0..296 the values mod 256, byte 297 = move_count >> 8, 298-299 zero)."""
    out[:, :297] = (obs & 0xFF).to(torch.uint8)
    out[:, 297] = ((obs[:, 295] >> 8) & 0xFF).to(torch.uint8)
    out[:, 298:] = 0
    return out


class DualStepVectorEnv:
    def __init__(self, num_envs, device=None, opponent="random", policy_seed=0, refill_period=None, table0=0,
                 opponent_obs=True, random_starts=False, step_counter=None, agent_obs_u8=False):
        """step_counter: optional int64 [1] device tensor that every dual_step increments by one in its
        last launch (spl_dual_io_t.step_counter) — a graph-captured rollout loop passes it to the
        agent's act as ply_base, so each replay draws fresh actions without a counter launch.
        agent_obs_u8: keep `self.agent_obs_u8`, uint8 [n, 300], the compact rows (spl_step_args_t.obs_u8)
        of the agent's observation, written by the opponent's step beside the int32 obs it returns
        (ABI 8): a fused actor reads a quarter of the bytes (FusedActorCritic.act accepts them)."""
        if isinstance(opponent, str) and opponent not in _DEVICE_POLICIES:
            raise ValueError(f"unknown device opponent {opponent!r}; choose {sorted(_DEVICE_POLICIES)} or a callable")
        if step_counter is not None and not (step_counter.dtype == torch.int64 and step_counter.numel() == 1):
            raise ValueError("step_counter must be an int64 [1] tensor on the env's device")
        self.eng = Engine(num_envs, 2, device=device, refill_period=refill_period, table0=table0)
        self.num_envs, self.device = num_envs, self.eng.device
        if step_counter is not None and step_counter.device != self.device:
            self.eng.close()
            raise ValueError("step_counter must be an int64 [1] tensor on the env's device")
        self.opponent = opponent
        self.policy_seed = int(policy_seed)
        self.want_opp_obs = opponent_obs
        t = torch
        n, dev = num_envs, self.device
        z = lambda dt: t.zeros(n, dtype=dt, device=dev)
        self.opp_actions = z(t.int32)
        # phase A (agent move) small outputs, kept apart from the engine's (phase B) buffers
        self.small_a = (z(t.float32), z(t.uint8), z(t.uint8), z(t.int8))
        self.agent_reward, self.opp_reward = z(t.float32), z(t.float32)
        self.done, self.game_ended_on, self.info_flags = z(t.bool), z(t.int8), z(t.uint8)  # done: 0/1 bytes
        self.opp_obs = t.zeros(n, _native.OBS_DIM, dtype=t.int32, device=dev) if opponent_obs else None
        self.agent_obs_u8 = t.zeros(n, _native.OBS_U8, dtype=t.uint8, device=dev) if agent_obs_u8 else None
        self.random_starts = bool(random_starts)
        from .fused_policy import OpponentPool
        self.pool = opponent if isinstance(opponent, OpponentPool) else None
        if self.pool is not None:  # per-table opponent of the current episode, and each table's episode count
            self.opp_group = z(t.int32)
            self.episode = z(t.int32)
            self.ep_opp = z(t.int32)  # info["episode_opponent_index"]: the opponent before this step's draw
            self.pool.track(self.opp_group)  # slots still in play are not overwritten by add_snapshot
        # the agent's move writes the opponent's observation as compact bytes for a fused fp32 opponent
        # (the pool kernel, FusedActorCritic.opponent(): Engine.step obs_u8): a quarter of the int32
        # rows' bytes to store and to read back
        self.opp_obs_u8 = None
        if self.pool is not None or getattr(opponent, "accepts_u8", False):
            self.opp_obs_u8 = t.zeros(n, _native.OBS_U8, dtype=t.uint8, device=dev)
        e = self.eng
        ra, ta, fa, wa = self.small_a
        p = lambda x: None if x is None else x.data_ptr()
        self._io = _native.DualIo(reward_a=p(ra), reward_b=p(e.reward), terminated_a=p(ta),
                                  terminated_b=p(e.terminated), flags_a=p(fa), flags_b=p(e.flags), winner_a=p(wa),
                                  winner_b=p(e.winner), agent_reward=p(self.agent_reward),
                                  opp_reward=p(self.opp_reward), done=p(self.done),
                                  game_ended_on=p(self.game_ended_on), info_flags=p(self.info_flags),
                                  obs=p(e.obs), final_obs=p(e.final_obs), opp_obs=p(self.opp_obs),
                                  step_counter=p(step_counter))
        self._step_counter = step_counter  # the launches point at it
        self._ply = 0

    # ------------------------------------------------------------------------------------
    def reset(self, seed=None, seeds=None):
        """Deal every table (env i seeded with seed + i, or seeds[i]; neither: continue each
        table's stream).  A fresh deal has player 0 to play, so the reference's opening loop never
        moves the opponent here (dual_step_native.py:60-77)."""
        if seeds is None and seed is not None:
            seeds = range(int(seed), int(seed) + self.num_envs)
        obs, mask = self.eng.reset(seeds=seeds)
        if self.agent_obs_u8 is not None:  # the compact rows of the fresh deals (the reset writes int32 rows)
            compact_rows(obs, self.agent_obs_u8)
        info = {"action_mask": mask, "to_play": obs[:, 294]}
        if self.pool is not None:  # every table starts an episode: draw its opponent
            self.pool.draw(self.opp_group, self.episode, None, self.eng.table0)
            info["opponent_index"] = self.opp_group
        return obs, info

    def dual_step(self, actions):
        """wrappers/dual_step_native.py:90-193 on every table: spl_step (agent) -> opponent
        actions -> spl_step (opponent, autoreset 2, gated by the agent's move in the same launch) ->
        spl_dual_finish."""
        e, lib = self.eng, self.eng.lib
        device_opp = isinstance(self.opponent, str)
        self._ply += 1
        ra, ta, fa, wa = self.small_a
        # phase A: the agent's move (no reset); a device opponent's reply is drawn in the same kernel
        e.step(actions, autoreset=False, final_obs=False, small=self.small_a,
               next_actions=self.opp_actions if device_opp else None,
               policy=_DEVICE_POLICIES[self.opponent] if device_opp else 0,
               policy_seed=self.policy_seed, ply=self._ply,
               obs_u8=None if device_opp else self.opp_obs_u8)
        if device_opp:
            opp = self.opp_actions
        elif self.pool is not None:
            opp = self.pool.act(self.opp_obs_u8, e.mask, self.opp_group, out=self.opp_actions)
        else:
            opp = self.opponent(e.obs if self.opp_obs_u8 is None else self.opp_obs_u8, e.mask)
            if not (isinstance(opp, torch.Tensor) and opp.dtype == torch.int32 and opp.is_contiguous()
                    and opp.device == self.device):
                opp = torch.as_tensor(opp, device=self.device).to(torch.int32).contiguous()
            self._opp_keep = opp
        stream = e.stream()
        with torch.cuda.device(self.device):
            # phase B: the opponent's move, gated in the same launch (-1, no move, where the agent's move
            # was not applied or ended the game); autoreset 2 also re-deals the tables that ended on
            # the agent's move
            e.step(opp, autoreset=2, final_obs=True, gate=(ta, fa), obs_u8=self.agent_obs_u8,
                   keep_obs=self.agent_obs_u8 is not None)
            io = self._io
            io.opp_obs = self.opp_obs.data_ptr() if self.want_opp_obs else None
            if self.pool is not None:  # finish + the finished tables' next-opponent draw, one launch
                self.pool.finish_draw(io, self.opp_group, self.episode, self.ep_opp, self.eng.table0)
            else:
                _native.check(lib, lib.spl_dual_finish(self.num_envs, ctypes.byref(io), stream))
        base = {"action_mask": e.mask, "to_play": e.obs[:, 294], "final_observation": e.final_obs,
                "opponent_action": opp, "game_ended_on": self.game_ended_on, "agent_step_reward": ra}
        if self.pool is not None:
            # the opponent that played this step's episode, then the next episode's for re-dealt tables
            base["episode_opponent_index"] = self.ep_opp
            base["opponent_index"] = self.opp_group
        info = DualInfo(base, self.info_flags)
        return e.obs, self.agent_reward, self.opp_obs, self.opp_reward, self.done, info

    def close(self):
        if self.pool is not None:
            self.pool.untrack(self.opp_group)
        self.eng.close()
