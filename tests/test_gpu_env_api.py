"""The reference's own env tests, run against the drop-in SplendorEnv / SplendorVectorEnv on the
GPU (reference tests: splendor_gym/tests/test_env.py, test_gym_compat.py, test_draw_rule.py,
test_take_reduced_colors.py, test_reserved_card_observation.py, test_properties.py,
test_afford_nobles_obs.py, test_rules.py), plus single-env parity against the oracle."""
import time

import numpy as np
import pytest

from oracle.oracle import Oracle, OracleVec

pytestmark = pytest.mark.gpu


def make_env():
    from splendor_gym.envs import SplendorEnv
    return SplendorEnv(num_players=2)


def first_legal(mask):
    return int(np.flatnonzero(mask)[0])


def test_reset_and_step_shapes():  # test_env.py:8-25, test_gym_compat.py:18-41
    env = make_env()
    obs, info = env.reset(seed=123)
    assert isinstance(obs, np.ndarray) and obs.shape == (297,) and obs.dtype == np.int32
    assert info["action_mask"].shape == (45,) and info["action_mask"].dtype == np.int8
    assert env.action_space.n == 45 and env.observation_space.shape == (297,)
    obs, r, term, trunc, info = env.step(first_legal(info["action_mask"]))
    assert isinstance(r, float) and isinstance(term, bool) and isinstance(trunc, bool)
    assert obs.shape == (297,) and "action_mask" in info


def test_random_rollout_no_crash():  # test_env.py:28-37
    env = make_env()
    obs, info = env.reset(seed=0)
    rs = np.random.default_rng(0)
    for _ in range(200):
        if info["action_mask"].sum() == 0:
            break
        obs, r, term, trunc, info = env.step(int(rs.choice(np.flatnonzero(info["action_mask"]))))
        if term:
            obs, info = env.reset()


def test_deterministic_reset_and_scripted_prefix():  # test_gym_compat.py:44-76, test_properties.py:23-36
    e1, e2 = make_env(), make_env()
    o1, i1 = e1.reset(seed=999)
    o2, i2 = e2.reset(seed=999)
    np.testing.assert_array_equal(o1, o2)
    for _ in range(20):
        a1, a2 = first_legal(i1["action_mask"]), first_legal(i2["action_mask"])
        assert a1 == a2
        o1, r1, t1, _, i1 = e1.step(a1)
        o2, r2, t2, _, i2 = e2.step(a2)
        np.testing.assert_array_equal(o1, o2)
        assert (r1, t1) == (r2, t2)


def test_step_after_terminated_raises():  # test_gym_compat.py:89-108
    env = make_env()
    obs, info = env.reset(seed=123)
    for _ in range(2000):
        m = info["action_mask"]
        obs, r, term, trunc, info = env.step(first_legal(m) if m.any() else 0)
        if term:
            break
    assert term
    with pytest.raises(RuntimeError):
        env.step(0)
    assert env.get_final_rewards() in ({0: 1.0, 1: -1.0}, {0: -1.0, 1: 1.0}, {0: 0.0, 1: 0.0}, {0: -0.1, 1: -0.1})


def test_illegal_action_penalty_and_oob():  # test_gym_compat.py:111-124, splendor_env.py:62-66
    env = make_env()
    obs, info = env.reset(seed=321)
    illegal = int(np.flatnonzero(info["action_mask"] == 0)[0])
    obs2, r, term, trunc, info2 = env.step(illegal)
    assert r == pytest.approx(-0.01) and not term and info2.get("illegal_action")
    np.testing.assert_array_equal(obs, obs2)
    with pytest.raises(ValueError):
        env.step(45)
    with pytest.raises(ValueError):
        env.step(-1)


def test_render_no_crash(capsys):  # test_gym_compat.py:127-132
    env = make_env()
    env.render_mode = "human"
    env.reset(seed=0)
    env.render()
    assert "Bank" in capsys.readouterr().out


def mask_from_state(env):  # reference tests/utils.py:15-16
    from splendor_gym.engine import legal_moves
    return np.array(legal_moves(env.state), dtype=np.int8)


def test_no_legal_move_draw():  # test_draw_rule.py:7-24, in-place edits of env.state (no set_state)
    """The reference resets from entropy (SplendorEnv(seed=0) does not seed reset) and reserves the
    first three tier-1 deck cards: when one of them costs white only, 10 white tokens buy it and its
    assertion fails (a flaky case of the reference test).  Here the reset is seeded with the first
    seed whose three cards are not all-white, which is the situation the test means."""
    from splendor_gym.envs import SplendorEnv
    env = SplendorEnv(seed=0)
    for seed in range(100):
        obs, info = env.reset(seed=seed)
        if not any(set(c for c, v in card.cost.items() if v) <= {"white"} for card in env.state.decks[1][:3]):
            break
    env.state.bank[:] = [0, 0, 0, 0, 0, 0]
    p = env.state.players[env.state.to_play]
    p.tokens[:] = [10, 0, 0, 0, 0, 0]
    p.reserved = env.state.decks[1][:3]
    for t in (1, 2, 3):
        env.state.board[t] = [None, None, None, None]
    assert not np.any(mask_from_state(env))
    assert not env.legal_mask().any()
    obs, reward, terminated, truncated, info = env.step(0)
    assert terminated and reward == 0 and info.get("draw") and env.state.winner_index is None


def test_take_two_when_only_two_colors():  # test_take_reduced_colors.py:7-21
    from splendor_gym.engine.state import COLOR_INDEX
    env = make_env()
    env.reset(seed=123)
    env.state.bank[:] = [0, 0, 0, 0, 0, 0]
    env.state.bank[COLOR_INDEX["white"]] = 1
    env.state.bank[COLOR_INDEX["green"]] = 2
    m = mask_from_state(env)
    legal = [i for i in range(0, 10) if m[i] == 1]
    assert legal == [0, 3, 4]
    env.step(legal[0])
    last = env.state.players[(env.state.to_play - 1) % env.state.num_players]
    assert last.tokens[COLOR_INDEX["white"]] + last.tokens[COLOR_INDEX["green"]] == 2


def test_take_one_when_only_one_color():  # test_take_reduced_colors.py:24-36
    from splendor_gym.engine.state import COLOR_INDEX
    env = make_env()
    env.reset(seed=123)
    env.state.bank[:] = [0, 0, 0, 0, 0, 0]
    env.state.bank[COLOR_INDEX["black"]] = 3
    m = mask_from_state(env)
    legal = [i for i in range(0, 10) if m[i] == 1]
    assert legal == [2, 4, 5, 7, 8, 9]
    env.step(legal[0])
    last = env.state.players[(env.state.to_play - 1) % env.state.num_players]
    assert last.tokens[COLOR_INDEX["black"]] == 1


def test_token_return_behavior_random_non_gold():  # test_afford_nobles_obs.py:58-71
    env = make_env()
    obs, info = env.reset(seed=7)
    state = env.state
    p = state.players[state.to_play]
    p.tokens = [3, 3, 3, 3, 3, 0]
    prev_bank = list(state.bank)
    env.step(int(np.flatnonzero(info["action_mask"])[0]))
    prev = env.state.players[(env.state.to_play - 1) % env.state.num_players]
    assert sum(prev.tokens) == 10 and sum(env.state.bank) >= sum(prev_bank)


def test_state_view_edits_match_the_oracle():
    """An edited env.state steps exactly like the same state in the CPU oracle."""
    from oracle.oracle import Oracle, table_to_view
    o = Oracle()
    env = make_env()
    env.reset(seed=11)
    s = env.state
    s.players[0].tokens[:] = [2, 2, 2, 2, 1, 1]
    s.bank[:] = [2, 2, 2, 2, 3, 4]
    s.players[0].bonuses[:] = [1, 0, 2, 0, 1]
    view = table_to_view(s.to_record())
    for a in range(45):
        if mask_from_state(env)[a]:
            break
    obs, r, term, trunc, info = env.step(a)
    ref = o.env_step(view, a)
    np.testing.assert_array_equal(obs, ref["obs"])
    from schema import canon
    assert canon(table_to_view(env.state.to_record())) == canon(ref["after"])


def test_render_text_matches_reference(capsys):  # envs/splendor_env.py:119-126 -> game_logger.py:159-220
    import json
    import os
    with open(os.path.join(os.path.dirname(__file__), "golden", "render.json")) as f:
        cases = json.load(f)["env"]
    for c in cases:
        env = make_env()
        env.reset(seed=c["seed"])
        for a in c["actions"]:
            env.step(a)
        capsys.readouterr()
        env.render()
        assert capsys.readouterr().out == c["text"], c["seed"]


def test_functional_engine_api_matches_reference():
    """engine.initial_state / legal_moves / apply_action / encode_observation on host views
    (evaluated on the GPU) against the reference's deals (deals.npz), legal masks of 148 logged
    states (render.json) and crafted/fuzzed steps (edge_cases.json)."""
    import json
    import os
    from oracle.oracle import table_to_view, view_to_table
    from splendor_gym.engine import apply_action, initial_state, legal_moves
    from splendor_gym.engine.encode import encode_observation
    from splendor_gym.engine.state import SplendorState
    gold = os.path.join(os.path.dirname(__file__), "golden")
    d = np.load(os.path.join(gold, "deals.npz"))
    for P in (2, 3, 4):
        for i in range(0, 512, 37):
            v = table_to_view(initial_state(P, int(d["seeds"][i])).to_record())
            assert v["board"] == [int(x) for x in d[f"board_p{P}"][i]]
            for t in range(3):
                dk = [int(x) for x in d[f"decks_p{P}"][i, t] if x >= 0]
                assert v["decks"][t] == dk
            assert v["nobles"] == [int(x) for x in d[f"nobles_p{P}"][i] if x >= 0]
    with open(os.path.join(gold, "render.json")) as f:
        states = json.load(f)["states"]
    for c in states:
        s = SplendorState.from_record(view_to_table(c["view"]))
        assert legal_moves(s) == c["mask"], c["name"]
    with open(os.path.join(gold, "edge_cases.json")) as f:
        cases = json.load(f)
    done = 0
    for c in cases:
        if c["exception"] is not None or c["flags"] != 0 or not (c["legal"] >> c["action"]) & 1:
            continue
        s = SplendorState.from_record(view_to_table(c["before"]))
        nxt = apply_action(s, c["action"])
        got = table_to_view(nxt.to_record())
        want = table_to_view(view_to_table(c["after"]))
        for p in got["players"] + want["players"]:
            p["nobles"] = sorted(p["nobles"])
        assert got == want, c["name"]
        np.testing.assert_array_equal(encode_observation(nxt), np.array(c["obs"], np.int32), err_msg=c["name"])
        assert s.to_record().tobytes() == view_to_table(c["before"]).tobytes()  # input not modified
        done += 1
    assert done > 300
    s = initial_state(2, 0)
    with pytest.raises(ValueError):
        apply_action(s, 45)
    with pytest.raises(ValueError):
        apply_action(s, 15)  # buying a card with no tokens: illegal


def test_reserved_card_visibility():  # test_reserved_card_observation.py:85-371
    env = make_env()
    obs, info = env.reset(seed=42)
    a = [i for i in range(27, 39) if info["action_mask"][i]][0]
    obs, _, _, _, info = env.step(a)                     # P0 reserves a visible card
    assert obs[18] == 0 and obs[31] == 1                  # P1 to play: own 0, opponent 1
    assert obs[230] == 1 and obs[230 + 13] == 1           # revealed to the opponent
    obs, _, _, _, info = env.step(first_legal(info["action_mask"]))  # P1 any move
    obs, _, _, _, info = env.step(39)                     # P0 blind-reserves tier 1
    assert obs[31] == 2 and obs[230 + 14:230 + 28].sum() == 0   # hidden slot is all zeros
    assert obs[230] == 1                                   # the visible one still shows


def test_mask_invariants():  # test_properties.py:39-57
    env = make_env()
    obs, info = env.reset(seed=7)
    s, m = env.state, info["action_mask"]
    for c in range(5):
        assert (m[10 + c] == 1) == (s.bank[c] >= 4)
    p = s.players[s.to_play]
    for t in (1, 2, 3):
        assert (m[38 + t] == 1) == (len(s.decks[t]) > 0 and len(p.reserved) < 3)


def test_token_return_to_ten():  # test_afford_nobles_obs.py:58-71, test_rules.py:37-43
    env = make_env()
    obs, info = env.reset(seed=7)
    s = env.state
    s.players[s.to_play].tokens = [3, 3, 3, 3, 3, 0]
    env.set_state(s)
    bank_before = sum(env.state.bank)
    env.step(first_legal(env.legal_mask()))
    s = env.state
    assert sum(s.players[(s.to_play - 1) % 2].tokens) == 10 and sum(s.bank) >= bank_before


def test_single_env_matches_oracle_with_stream_continuation():
    """SplendorEnv episodes (reset(seed) then reset() continuing the np_random stream) equal the
    oracle step for step."""
    orc = Oracle()
    env = make_env()
    vec = OracleVec(orc, 1, 2, [2024])
    obs, info = env.reset(seed=2024)
    np.testing.assert_array_equal(obs, vec.obs[0])
    rs = np.random.default_rng(5)
    episodes = 0
    while episodes < 3:
        legal = np.flatnonzero(info["action_mask"])
        a = int(rs.choice(legal)) if len(legal) else 0
        obs, r, term, trunc, info = env.step(a)
        ref = vec.step(np.array([a], np.int32), want_final=True)
        np.testing.assert_array_equal(obs, ref["final_obs"][0] if term else ref["obs"][0])
        assert np.float32(r) == ref["reward"][0]
        if term:
            episodes += 1
            obs, info = env.reset()
            np.testing.assert_array_equal(obs, ref["obs"][0])


def test_single_env_without_a_same_address_host_mapping_matches_oracle(monkeypatch):
    """SplendorEnv hands the kernels its pinned I/O block's host address only when
    spl_host_mapped says the device sees it at that address; otherwise (forced here) it steps through a
    device block with copies, with the same results as the oracle, masks and errors included."""
    from splendor_gym.device import Engine
    monkeypatch.setattr(Engine, "_host_mapped", lambda self, ptr: False)
    orc = Oracle()
    env = make_env()
    vec = OracleVec(orc, 1, 2, [77])
    obs, info = env.reset(seed=77)
    assert not env._eng.host_io and env._eng.io.is_cuda
    np.testing.assert_array_equal(obs, vec.obs[0])
    np.testing.assert_array_equal(env.legal_mask(), info["action_mask"])
    rs = np.random.default_rng(3)
    for _ in range(120):
        legal = np.flatnonzero(info["action_mask"])
        a = int(rs.choice(legal)) if len(legal) else 0
        obs, r, term, trunc, info = env.step(a)
        ref = vec.step(np.array([a], np.int32), want_final=True)
        np.testing.assert_array_equal(obs, ref["final_obs"][0] if term else ref["obs"][0])
        assert np.float32(r) == ref["reward"][0]
        if term:
            obs, info = env.reset()
            np.testing.assert_array_equal(obs, ref["obs"][0])
    with pytest.raises(ValueError):
        env.step(45)


def test_pinned_io_block_is_mapped_at_its_own_address():
    """The probe itself on this box: torch's pinned host allocator hands out hipHostMalloc memory that
    the device sees at the same address (so SplendorEnv takes the zero-copy path)."""
    env = make_env()
    env.reset(seed=1)
    e = env._eng
    assert e.host_io and e._host_mapped(e.io.data_ptr())


def test_vector_env_matches_single_envs_and_autoresets():
    import torch
    from splendor_gym import SplendorVectorEnv
    n = 8
    vec = SplendorVectorEnv(n, device="cuda:0")
    obs, info = vec.reset(seed=100)
    singles = [make_env() for _ in range(n)]
    for i, e in enumerate(singles):
        o, _ = e.reset(seed=100 + i)
        np.testing.assert_array_equal(obs[i].cpu().numpy(), o)
    saw_final = False
    for k in range(300):
        acts = vec.sample_actions(seed=3, ply=k).clone()
        obs, rew, term, trunc, info = vec.step(acts)
        for i, e in enumerate(singles):
            o, r, t, _, _ = e.step(int(acts[i]))
            if t:
                np.testing.assert_array_equal(info["final_observation"][i].cpu().numpy(), o)
                o, _ = e.reset()
                saw_final = True
            np.testing.assert_array_equal(obs[i].cpu().numpy(), o)
            assert np.float32(rew[i].item()) == np.float32(r) and bool(term[i]) == t
    assert saw_final


def test_vector_env_numpy_mode():
    from splendor_gym import SplendorVectorEnv
    vec = SplendorVectorEnv(16, device="cuda:0", to_numpy=True)
    obs, info = vec.reset(seed=0)
    assert isinstance(obs, np.ndarray) and obs.shape == (16, 297) and info["action_mask"].shape == (16, 45)
    done = 0
    for k in range(400):
        acts = vec.sample_actions(seed=1, ply=k).cpu().numpy()
        obs, rew, term, trunc, info = vec.step(acts)
        if term.any():
            i = int(np.flatnonzero(term)[0])
            assert info["_final_observation"][i] and info["final_observation"][i].shape == (297,)
            assert "final_rewards" in info["final_info"][i]
            done += 1
    assert done > 0


def test_vector_env_action_errors():
    """Out-of-range actions raise the reference's ValueError (envs/splendor_env.py:63-64): host
    arrays are checked before the launch, device tensors by the step itself ("sync") or by the
    next call ("deferred"); info's flag views follow the per-table flags."""
    import torch
    from splendor_gym import SplendorVectorEnv
    from splendor_gym import _native
    n = 64
    for mode in ("sync", "deferred"):
        vec = SplendorVectorEnv(n, device="cuda:0", check_actions=mode)
        vec.reset(seed=7)
        bad = np.zeros(n, np.int32)
        bad[5] = 45
        with pytest.raises(ValueError):
            vec.step(bad)  # host actions: before any launch
        acts = vec.sample_actions(seed=2, ply=0).clone()
        obs, rew, term, trunc, info = vec.step(acts)
        fl = vec.last_flags
        assert torch.equal(info["illegal_action"], (fl & _native.F_ILLEGAL) != 0)
        assert torch.equal(info["draw"], (fl & _native.F_DRAW) != 0)
        assert torch.equal(info["turn_limit"], (fl & _native.F_TURN_LIMIT) != 0)
        assert term.dtype == torch.bool and not trunc.any()
        dev_bad = vec.sample_actions(seed=2, ply=1).clone()
        dev_bad[9] = -1
        if mode == "sync":
            with pytest.raises(ValueError, match="envs \\[9\\]"):
                vec.step(dev_bad)
        else:
            vec.step(dev_bad)  # returns; the error comes back with a later call
            with pytest.raises(ValueError, match="deferred"):
                for k in range(vec.DEFER_EVERY * (vec.DEFER_LAG + 1)):
                    vec.step(vec.sample_actions(seed=2, ply=2 + k).clone())
            vec.step(dev_bad)
            with pytest.raises(ValueError, match="deferred"):
                vec.reset(seed=8)  # reset() waits for every pending check
        vec.close()


def test_vector_env_returns_fresh_arrays_while_held():
    """copy=True (gymnasium SyncVectorEnv's default): what a step returned is not overwritten by later
    steps while the caller holds it (the old step() returned buffers the next step
    overwrote); copy=False returns the same buffers every step."""
    import torch
    from splendor_gym import SplendorVectorEnv
    n = 256
    vec = SplendorVectorEnv(n, device="cuda:0")
    vec.reset(seed=3)
    held = []
    for k in range(6):
        obs, rew, term, trunc, info = vec.step(vec.sample_actions(seed=4, ply=k).clone())
        snap = [t.clone() for t in (obs, rew, term, trunc, info["action_mask"], info["illegal_action"],
                                    info["to_play"], info["final_observation"])]
        held.append(((obs, rew, term, trunc, info["action_mask"], info["illegal_action"], info["to_play"],
                      info["final_observation"]), snap))
    row = held[0][0][0][7]  # a view into the first step's obs, the tuple dropped below
    row_snap = row.clone()
    for live, snap in held:
        for a, b in zip(live, snap):
            assert torch.equal(a, b)
    held.clear()
    for k in range(6, 12):
        vec.step(vec.sample_actions(seed=4, ply=k).clone())
    assert torch.equal(row, row_snap)  # a view keeps its block alive
    # dropped results are recycled: the ring does not grow without bound
    assert len(vec._ring) <= vec.RING + 1
    vec.close()
    alias = SplendorVectorEnv(n, device="cuda:0", copy=False)
    alias.reset(seed=3)
    a = alias.step(alias.sample_actions(seed=4, ply=0).clone())
    b = alias.step(alias.sample_actions(seed=4, ply=1).clone())
    assert a[0].data_ptr() == b[0].data_ptr() and not b[3].any()
    alias.close()


@pytest.mark.slow
def test_rollout_perf_smoke():  # test_gym_compat.py:135-157 (threshold 6000 SPS)
    env = make_env()
    obs, info = env.reset(seed=123)
    n, steps = 5000, 0
    t0 = time.time()
    while steps < n:
        m = info["action_mask"]
        obs, r, term, trunc, info = env.step(first_legal(m) if m.any() else 0)
        steps += 1
        if term:
            obs, info = env.reset(seed=steps)
    sps = steps / (time.time() - t0)
    print(f"SPS={sps:.0f}")
    assert sps > 6000


def test_engine_rules_reference_cases():  # test_rules.py:8-43, test_afford_nobles_obs.py:31-55
    from splendor_gym.engine import apply_action, initial_state, legal_moves
    from splendor_gym.engine.encode import OBSERVATION_DIM, TOTAL_ACTIONS, encode_observation
    s = initial_state(seed=42)
    m = legal_moves(s)
    assert len(m) == TOTAL_ACTIONS and any(m)
    s = initial_state(seed=1)
    a = next(i for i, v in enumerate(legal_moves(s)) if v == 1)
    nxt = apply_action(s, a)
    assert sum(nxt.bank) == sum(s.bank) - (3 if a < 10 else 2 if a < 15 else 0)
    assert nxt.turn_count == s.turn_count
    s = initial_state(seed=0)
    m = legal_moves(s)
    assert all(m[10 + c] == 0 for c in range(5) if s.bank[c] < 4)
    s.players[s.to_play].tokens = [5, 5, 5, 5, 5, 0]  # token return seeded outside the table's domain
    nxt = apply_action(s, 0)
    assert sum(nxt.players[s.to_play - 1].tokens) <= 10
    s = initial_state(seed=999)
    s.players[s.to_play].bonuses = [4, 4, 4, 4, 4]
    nxt = apply_action(s, int(np.flatnonzero(legal_moves(s))[0]))
    assert sum(1 for n in nxt.nobles if n is None) == 1  # exactly one noble per turn
    obs = encode_observation(initial_state(seed=0))
    assert obs.shape == (OBSERVATION_DIM,) and obs.dtype == np.int32


def test_affordability_with_an_edited_card_cost():  # test_afford_nobles_obs.py:9-28
    """The reference test edits a board card's cost in place (card.cost = {...}); the functional API
    evaluates that state on a context built from the state's card table."""
    from splendor_gym.engine import apply_action, initial_state, legal_moves
    from splendor_gym.engine.state import COLOR_INDEX
    state = initial_state(seed=123)
    p = state.players[state.to_play]
    p.tokens = [0, 1, 0, 1, 0, 1]  # one blue, one red, one gold
    p.bonuses = [0, 0, 0, 1, 0]    # one red bonus
    card = state.board[1][0]
    card.cost = {"red": 2, "blue": 2}
    state.bank = [4, 4, 4, 4, 4, 5]
    mask = legal_moves(state)
    assert mask[15] == 1  # buy tier-1 slot 0: red 2-1 bonus = 1 token, blue 2 = 1 token + 1 gold
    nxt = apply_action(state, 15)
    prev = nxt.players[(nxt.to_play - 1) % nxt.num_players]
    assert prev.tokens[COLOR_INDEX["gold"]] <= 1
    assert all(t >= 0 for t in prev.tokens)
    # exactly what the edited cost implies (state.py:61-71 + rules.py:101-115): all tokens spent
    assert prev.tokens == [0, 0, 0, 0, 0, 0]
    assert nxt.bank == [4, 5, 4, 5, 4, 6]
    assert all(c is None or c.id != card.id for c in nxt.board[1])  # the edited card left the board
    # the same buy is illegal with the card's canonical cost whenever that cost is not coverable
    from splendor_gym.engine.state import cards_by_id
    canon = cards_by_id()[card.id]
    base_need = sum(max(0, canon.cost.get(c, 0) - b) for c, b in zip(("white", "blue", "green", "red", "black"),
                                                                       p.bonuses))
    if base_need > 3:
        state.board[1][0] = type(card)(canon.id, canon.tier, canon.color, canon.points, dict(canon.cost))
        assert legal_moves(state)[15] == 0


def test_edited_card_cost_through_the_env_and_the_oracle():
    """The same edit through SplendorEnv.state (write-through): the env switches to the edited card
    table for the episode; legal mask, step outputs and the next observation equal the CPU oracle
    evaluating the edited card table (oracle/splendor_oracle.c with its own card table)."""
    from splendor_gym.envs import SplendorEnv
    env = SplendorEnv()
    obs, info = env.reset(seed=31)
    s = env.state
    p = s.players[s.to_play]
    p.tokens = [0, 1, 0, 1, 0, 1]
    p.bonuses = [0, 0, 0, 1, 0]
    card = s.board[1][0]
    card.cost = {"red": 2, "blue": 2}
    s.bank = [4, 4, 4, 4, 4, 5]
    tbl, rec = s.card_table(), s.to_record()
    assert tbl is not None and list(tbl[card.id][3:]) == [0, 2, 0, 2, 0]
    m = env.legal_mask()
    assert m[15] == 1
    obs2, r, term, trunc, info2 = env.step(15)
    assert r == 0.0 and not term and info2["action_mask"].shape == (45,)
    # the CPU oracle on the same edited card table (orc_set_tables), restored afterwards
    from oracle.oracle import Oracle, table_to_view
    orc = Oracle()
    orc.L.orc_set_tables(np.ascontiguousarray(tbl).ctypes.data, orc.nobles.ctypes.data)
    try:
        view = table_to_view(rec)
        ref_mask = orc.legal(view)
        ref = orc.env_step(view, 15)
    finally:
        orc.L.orc_set_tables(orc.cards.ctypes.data, orc.nobles.ctypes.data)
    assert int((m.astype(np.uint64) << np.arange(45, dtype=np.uint64)).sum()) == ref_mask
    assert not ref["error"] and np.array_equal(obs2, ref["obs"]) and np.float32(r) == np.float32(ref["reward"])
    assert int((info2["action_mask"].astype(np.uint64) << np.arange(45, dtype=np.uint64)).sum()) == ref["mask"]
    after = env.state
    assert after.players[0].tokens == [0, 0, 0, 0, 0, 0] and after.players[0].bonuses[STD.index(card.color)] >= 1
    assert after.bank == [4, 5, 4, 5, 4, 6]
    # the edited object stays the episode's card: a later view shows the edited cost wherever it is
    assert all(c.cost == {"red": 2, "blue": 2} for c in after.cards().values() if c.id == card.id)
    obs_r, info_r = env.reset(seed=31)  # a new game deals canonical cards again
    assert env.state.card_table() is None
    # ... and the reset's own obs/mask come from the canonical table: the edited card
    # is dealt to the same slot again, so an obs built from the old context would show its edit
    fresh = SplendorEnv()
    obs_f, info_f = fresh.reset(seed=31)
    assert np.array_equal(obs_r, obs_f) and np.array_equal(info_r["action_mask"], info_f["action_mask"])
    assert np.array_equal(obs_r, obs)


STD = ["white", "blue", "green", "red", "black"]
