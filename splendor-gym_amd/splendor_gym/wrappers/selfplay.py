"""SelfPlayWrapper: the agent is player 0; player 1's moves are played by an opponent policy
inside reset/step.  Drop-in for reference splendor_gym/wrappers/selfplay.py:5-73."""
from .._gym_compat import Wrapper
from ._common import episode_opponent, play_opening, random_opponent  # noqa: F401


class SelfPlayWrapper(Wrapper):
    def __init__(self, env, opponent_policy, random_starts: bool = True, opponent_supplier=None):
        super().__init__(env)
        self.opponent_policy = opponent_policy
        self.random_starts = random_starts
        self.opponent_supplier = opponent_supplier
        self._opp_policy = opponent_policy

    def reset(self, **kwargs):
        self._opp_policy = episode_opponent(self)  # selfplay.py:20-25
        obs, info = self.env.reset(**kwargs)
        return play_opening(self, obs, info)

    def step(self, action):
        """Agent move, then (unless the game ended) one opponent move.  Reward from player 0's
        side: the agent's own terminal reward, minus the opponent's when its move ends the game,
        else 0 (selfplay.py:42-63)."""
        obs, reward, term, trunc, info = self.env.step(action)
        if term or trunc:
            return obs, reward, term, trunc, info
        if info.get("to_play", 0) != 1:
            raise RuntimeError(
                f"Invalid state: game not terminal but to_play={info.get('to_play', 'unknown')} (expected 1 for opponent)")
        obs, opp_reward, term, trunc, info = self.env.step(self._opp_policy(obs, info))
        return obs, (-opp_reward if (term or trunc) else 0.0), term, trunc, info
