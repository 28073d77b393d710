"""CPU tests of the drop-in host surface (no GPU): the reference trainer's imports, signatures of
the re-implemented modules, the game logger's text against the reference (tests/golden/render.json)
and the reference-signature evaluation loop against tests/golden/eval.json on the oracle env double."""
import inspect
import json
import os

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

# The import statements of the reference trainer (ppo_splendor.py:10-24) and of the reference
# training_utils.py (:20-28), as data.  `import gymnasium as gym` (ppo_splendor.py:4) is the
# user's own dependency and is not installed in this image.
PPO_IMPORT_LINES = [
    "from splendor_gym.engine.encode import OBSERVATION_DIM, TOTAL_ACTIONS",
    "from splendor_gym.scripts.eval_suite import (model_greedy_policy_from, random_opponent, "
    "greedy_opponent_v1, basic_priority_opponent)",
    "from training_utils import (TrainingLogger, CheckpointManager, make_env, run_evaluation_suite, "
    "frozen_policy_from, linear_lr_schedule)",
    "from splendor_gym.envs import SplendorEnv",
    "from splendor_gym.wrappers.selfplay import SelfPlayWrapper, random_opponent",
    "from splendor_gym.scripts.eval_suite import (eval_vs_opponent, model_greedy_policy_from, "
    "make_selfplay_env_with, greedy_opponent_v1, basic_priority_opponent)",
    "from splendor_gym.wrappers.dual_step_native import DualStepNativeWrapper",
    "from splendor_gym.wrappers.dual_step_selfplay import DualStepSelfPlayWrapper",
    # engine API of the reference tests and game logger (engine/__init__.py:1-13)
    "from splendor_gym.engine import SplendorState, legal_moves, apply_action, is_terminal, winner, initial_state",
    "from splendor_gym.engine.encode import OBSERVATION_DIM, encode_observation",
    "from splendor_gym.engine.state import COLOR_INDEX, STANDARD_COLORS, HUMAN_TO_INTERNAL",
    "from splendor_gym.scripts.game_logger import SplendorGameLogger, run_logged_game",
]

# parameter names of the reference functions (read from the reference sources)
SIGNATURES = {
    ("training_utils", "make_env"): ["seed", "opponent_policy", "opponent_supplier", "random_starts",
                                     "use_dual_step", "use_dual_player"],
    ("training_utils", "run_evaluation_suite"): ["agent", "device", "rng", "n_games", "update_seed"],
    ("training_utils", "frozen_policy_from"): ["state_dict", "actor_critic_class", "obs_dim", "act_dim", "device"],
    ("training_utils", "linear_lr_schedule"): ["initial_lr", "progress"],
    ("training_utils", "TrainingLogger"): ["log_dir", "track"],
    ("training_utils", "CheckpointManager"): ["log_dir", "run_start_ts"],
    ("splendor_gym.scripts.eval_suite", "eval_vs_opponent"): ["make_env", "model_policy", "n_games", "seed"],
    ("splendor_gym.scripts.eval_suite", "eval_vs_checkpoint_pool"): ["checkpoint_paths", "model_policy", "n_games",
                                                                    "seed"],
    ("splendor_gym.scripts.eval_suite", "make_selfplay_env_with"): ["opponent_policy", "seed"],
    ("splendor_gym.scripts.eval_suite", "model_greedy_policy_from"): ["model", "device"],
    ("splendor_gym.scripts.eval_suite", "greedy_opponent_v2_factory"): ["env_ref"],
    ("splendor_gym.engine", "initial_state"): ["num_players", "seed"],
    ("splendor_gym.engine", "apply_action"): ["state", "action"],
}


@pytest.mark.parametrize("line", PPO_IMPORT_LINES)
def test_reference_import_lines(line):
    exec(line, {})


@pytest.mark.parametrize("key", sorted(SIGNATURES))
def test_reference_signatures(key):
    import importlib
    mod, name = key
    obj = getattr(importlib.import_module(mod), name)
    params = list(inspect.signature(obj).parameters)
    assert params == SIGNATURES[key], (key, params)


def test_training_utils_without_tensorboard(tmp_path):
    import torch
    import training_utils as tu
    log = tu.TrainingLogger(str(tmp_path), track=True)  # tensorboard absent: no writer, no crash
    log.log_training_metrics(1, 1e-3, 0.1, 0.2, 0.3, 0.01)
    res = {k: {"win_rate": 0.5, "win_rate_ci95": 0.1, "avg_turns": 30.0, "draws": 1, "n": 4, "avg_prestige": 9.0}
           for k in ("random", "greedy_v1", "basic", "self_play")}
    log.log_evaluation_results(res, 1)
    log.update_history(1, res, 1e-3, 0.1, 0.2, 0.3)
    assert log.history.wr_basic == [0.5] and log.history.turns_self == [30.0]
    log.create_summary_plot(1)  # False without matplotlib
    cm = tu.CheckpointManager(str(tmp_path), log.run_start_ts)
    latest, stamped = cm.save_checkpoint(torch.nn.Linear(2, 2))
    assert os.path.exists(latest) and os.path.exists(stamped)
    assert tu.linear_lr_schedule(2.0, 0.25) == 0.5


def _render_fixture():
    with open(os.path.join(GOLD, "render.json")) as f:
        return json.load(f)


def test_game_logger_text_matches_reference():
    from oracle.oracle import view_to_table
    from splendor_gym.engine.state import SplendorState
    from splendor_gym.scripts.game_logger import SplendorGameLogger
    lg = SplendorGameLogger()
    cases = _render_fixture()["states"]
    assert len(cases) > 100
    for c in cases:
        s = SplendorState.from_record(view_to_table(c["view"]))
        assert lg.format_game_state(s) == c["text"], c["name"]
        assert [lg.decode_action(a, s) for a in range(45)] == c["actions"], c["name"]
        assert s.copy().to_record().tobytes() == s.to_record().tobytes()


def test_host_view_can_afford_and_editable_cards():
    from oracle.oracle import Oracle, view_to_table
    from splendor_gym.engine.state import SplendorState
    s = SplendorState.from_record(view_to_table(Oracle().initial_state(2, 3)))
    p = s.players[0]
    p.tokens = [0, 1, 0, 1, 0, 1]
    card = s.board[1][0]
    ok, need = p.can_afford(card)
    assert len(need) == 5 and ok == (sum(max(0, n - t) for n, t in zip(need, p.tokens)) <= 1)
    card.cost["red"] = 2  # editable per state, as the reference's (its card table follows)
    assert s.card_table()[card.id][6] == 2


@pytest.mark.parametrize("case", range(4))
def test_reference_signature_eval_on_oracle_env(case):
    """scripts.eval_suite.eval_vs_opponent (reference signature, one env per game) reproduces the
    reference's statistics (tests/golden/eval.json) on the oracle-backed env double."""
    from oracle_env import OracleSplendorEnv
    from splendor_gym.scripts.eval_suite import eval_vs_opponent, greedy_opponent_v1
    from splendor_gym.wrappers.selfplay import SelfPlayWrapper
    with open(os.path.join(GOLD, "eval.json")) as f:
        c = json.load(f)[case]

    def agent(obs, info):
        legal = np.flatnonzero(info["action_mask"])
        return int((legal[0] if c["agent"] == "first_legal" else legal[-1]) if len(legal) else 0)

    def make_env():
        env = SelfPlayWrapper(OracleSplendorEnv(), opponent_policy=greedy_opponent_v1)
        env.reset(seed=0)
        return env

    got = eval_vs_opponent(make_env, agent, n_games=c["n_games"], seed=c["seed"])
    want = c["result"]
    for k in ("n", "wins", "losses", "draws"):
        assert got[k] == want[k], (k, got, want)
    for k in ("win_rate", "win_rate_ci95", "avg_turns", "avg_prestige", "illegal_action_rate"):
        assert got[k] == pytest.approx(want[k], abs=1e-12), (k, got, want)
