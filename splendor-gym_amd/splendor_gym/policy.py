"""The reference's actor network and its action selection, batched for on-device self-play.

ActorCritic / masked_categorical restate ppo_splendor.py:27-59 (same layers and masking rule);
greedy_actions restates eval_suite.py:131-141 model_greedy_policy_from for a whole batch.
Weights here are whatever the caller loads; bench.py's config-5 line and tools/bench_selfplay.py load
the reference checkpoint (runs/ppo_splendor/ppo_splendor_latest.pt, committed as
tests/golden/ppo_splendor_latest.safetensors).
"""
import torch
import torch.nn as nn
from torch.distributions.categorical import Categorical

from .engine.encode import OBSERVATION_DIM, TOTAL_ACTIONS


def masked_categorical(logits: torch.Tensor, mask: torch.Tensor) -> Categorical:
    """Categorical over the legal actions; rows without a legal action keep their raw logits
    (the env reports the no-legal-move draw itself) (ppo_splendor.py:27-37).  Argument validation
    is off: it reads values back to the host, which a captured HIP graph cannot do."""
    illegal = mask < 0.5
    any_legal = (~illegal).any(dim=1, keepdim=True)
    return Categorical(logits=logits.masked_fill(illegal & any_legal, float("-inf")), validate_args=False)


class ActorCritic(nn.Module):
    """ppo_splendor.py:40-59: separate actor and critic MLPs, 297 -> 256 -> 256 -> (45 | 1), tanh."""

    def __init__(self, obs_dim: int = OBSERVATION_DIM, act_dim: int = TOTAL_ACTIONS):
        super().__init__()
        self.critic = nn.Sequential(nn.Linear(obs_dim, 256), nn.Tanh(), nn.Linear(256, 256), nn.Tanh(),
                                    nn.Linear(256, 1))
        self.actor = nn.Sequential(nn.Linear(obs_dim, 256), nn.Tanh(), nn.Linear(256, 256), nn.Tanh(),
                                   nn.Linear(256, act_dim))

    def get_value(self, x: torch.Tensor) -> torch.Tensor:
        return self.critic(x)

    def get_action_and_value(self, x: torch.Tensor, mask: torch.Tensor, action: torch.Tensor = None):
        probs = masked_categorical(self.actor(x), mask)
        if action is None:
            action = probs.sample()
        return action, probs.log_prob(action), probs.entropy().mean(), self.critic(x)


@torch.no_grad()
def greedy_actions(model: ActorCritic, obs: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
    """argmax of the actor's logits over legal actions, for every row (eval_suite.py:131-141)."""
    logits = model.actor(obs.float())
    return torch.argmax(logits.masked_fill(mask < 1, float("-inf")), dim=-1).to(torch.int32)


def greedy_opponent_from(model: ActorCritic):
    """A batched opponent for DualStepVectorEnv: (obs int32 [N,297], mask int8 [N,45]) -> int32 [N]."""
    model.eval()
    return lambda obs, mask: greedy_actions(model, obs, mask)
