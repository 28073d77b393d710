"""Generate the golden fixtures that pin the CPU oracle to the REAL reference engine.

Runs ONLY in the build container (it imports the read-only reference from /root/reference).
Nothing on the GPU box runs this; the outputs are committed under tests/golden/.

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

How the reference is loaded: a stub parent package ``splendor_gym`` whose
``__path__`` points at the reference (its real ``__init__`` imports gymnasium, which is not
installed), plus a minimal ``gymnasium`` stand-in that reproduces gymnasium 0.29's seeding
(``Env.reset(seed)`` -> ``Generator(PCG64(SeedSequence(seed)))``, later resets continue the
stream).  The stand-in is test scaffolding for the reference's env module only: the gymnasium
seeding boundary is therefore pinned to numpy's PCG64, not to a real gymnasium install
("parity unpinned" at that boundary).

Fixtures written (all small):
  mt_kat.npz      G1  CPython MT19937 / _randbelow / shuffle known answers
  deals.npz       G2  initial_state(P, seed) deck orders, boards, nobles, P in {2,3,4}
  seeding.npz     G4  env seed -> engine seed for reset(seed) + 4 continued resets
  traj_p{2,3,4}.npz G3 env trajectories (seeded random policy with ~3% illegal actions,
                      autoreset by reset() without seed) — per-ply action/reward/flags/obs
                      digests/mask/state digests, full obs for the first tables
  edge_cases.json G5  crafted states mirroring the reference tests + fuzzed states
"""
import hashlib
import json
import os
import random
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from schema import digest, from_ref_state  # noqa: E402

REF = "/root/reference"


# ----------------------------------------------------------------------------------------
# reference loading
# ----------------------------------------------------------------------------------------
def _install_gym_standin():
    gym = types.ModuleType("gymnasium")
    spaces = types.ModuleType("gymnasium.spaces")
    utils = types.ModuleType("gymnasium.utils")

    class Discrete:
        def __init__(self, n):
            self.n = n

    class Box:
        def __init__(self, low, high, shape, dtype):
            self.low, self.high, self.shape, self.dtype = low, high, shape, dtype

    class Env:
        _np_random = None

        def reset(self, *, seed=None, options=None):
            # gymnasium 0.29 Env.reset: reseed only when a seed is given
            if seed is not None:
                self._np_random = np.random.Generator(np.random.PCG64(np.random.SeedSequence(seed)))

        @property
        def np_random(self):
            if self._np_random is None:
                self._np_random = np.random.Generator(np.random.PCG64(np.random.SeedSequence(None)))
            return self._np_random

        def close(self):
            pass

    class Wrapper(Env):
        def __init__(self, env):
            self.env = env

    spaces.Discrete, spaces.Box = Discrete, Box
    gym.Env, gym.Wrapper, gym.spaces, gym.utils = Env, Wrapper, spaces, utils
    sys.modules["gymnasium"] = gym
    sys.modules["gymnasium.spaces"] = spaces
    sys.modules["gymnasium.utils"] = utils


def load_reference():
    _install_gym_standin()
    pkg = types.ModuleType("splendor_gym")
    pkg.__path__ = [os.path.join(REF, "splendor_gym")]
    sys.modules["splendor_gym"] = pkg
    import splendor_gym.engine as eng
    import splendor_gym.engine.encode as enc
    import splendor_gym.engine.rules as rules
    import splendor_gym.engine.state as st
    import splendor_gym.envs.splendor_env as envmod
    return eng, enc, rules, st, envmod


eng, enc, rules, st, envmod = load_reference()
CARDS = {c.id: c for t in (1, 2, 3) for c in st._load_cards_from_json()[t]}
NOBLES = {n.id - 1000: n for n in st._load_nobles_from_json()}


def make_env(P):
    env = envmod.SplendorEnv(num_players=2)
    env.num_players = P  # reference env refuses P != 2 in __init__ only; step logic is generic
    return env


def to_ref_state(v):
    """view -> reference SplendorState (fresh Card objects are shared from CARDS: never mutated)."""
    players = []
    for p in v["players"]:
        players.append(st.PlayerState(tokens=list(p["tokens"]), bonuses=list(p["bonuses"]),
                                      prestige=p["prestige"],
                                      reserved=[CARDS[i] for i in p["reserved"]],
                                      revealed_reserved=list(bool(x) for x in p["revealed"]),
                                      nobles=[NOBLES[i] for i in p["nobles"]]))
    board = {t: [(CARDS[v["board"][(t - 1) * 4 + s]] if v["board"][(t - 1) * 4 + s] >= 0 else None)
                 for s in range(4)] for t in (1, 2, 3)}
    decks = {t: [CARDS[i] for i in v["decks"][t - 1]] for t in (1, 2, 3)}
    nobles = [(NOBLES[i] if i >= 0 else None) for i in v["nobles"]]
    return st.SplendorState(num_players=v["P"], bank=list(v["bank"]), players=players, board=board,
                            decks=decks, nobles=nobles, to_play=v["to_play"],
                            turn_count=v["turn_count"], move_count=v["move_count"],
                            game_over=bool(v["game_over"]),
                            winner_index=(None if v["winner"] < 0 else v["winner"]),
                            turn_limit_reached=bool(v["turn_limit_reached"]))


def obs_digest(obs):
    return int.from_bytes(hashlib.blake2b(np.asarray(obs, dtype=np.int32).tobytes(),
                                          digest_size=8).digest(), "little")


def mask_bits(mask):
    m = 0
    for i, x in enumerate(mask):
        if x:
            m |= 1 << i
    return m


def info_flags(info):
    return (int(bool(info.get("illegal_action"))) | (int(bool(info.get("draw"))) << 1)
            | (int(bool(info.get("turn_limit"))) << 2))


# ----------------------------------------------------------------------------------------
# G1: MT19937 known answers
# ----------------------------------------------------------------------------------------
def gen_mt_kat():
    seeds = [0, 1, 2, 42, 12345, 2**31 - 2, 2**31 - 1, 2**32 - 1, 2**32, 2**32 + 5, 2**36 - 1,
             123456789012, 2**40 + 3]
    rs = random.Random(99)
    # token-return style seeds (engine/rules.py:170-175): the reachable domain and beyond
    for _ in range(256):
        tc, tp, stok, sbank = rs.randint(1, 101), rs.randint(0, 3), rs.randint(11, 28), rs.randint(0, 25)
        seeds.append((tc * 1315423911) ^ (tp * 2654435761) ^ (stok * 97531) ^ (sbank * 31337))
    words = np.zeros((len(seeds), 64), np.uint32)
    for i, s in enumerate(seeds):
        r = random.Random(s)
        words[i] = [r.getrandbits(32) for _ in range(64)]
    rb_n = np.array([1, 2, 3, 4, 5, 7, 10, 20, 30, 40], np.int64)
    rb = np.zeros((len(rb_n), 64), np.int64)
    for i, n in enumerate(rb_n):
        r = random.Random(7 + i)
        rb[i] = [r._randbelow(int(n)) for _ in range(64)]
    sh_n = [10, 20, 30, 40]
    shuf = np.full((len(sh_n), 64, 40), -1, np.int16)
    for i, n in enumerate(sh_n):
        for s in range(64):
            x = list(range(n))
            random.Random(s * 1000003 + n).shuffle(x)
            shuf[i, s, :n] = x
    np.savez_compressed(os.path.join(HERE, "mt_kat.npz"), seeds=np.array(seeds, np.uint64), words=words,
                        rb_n=rb_n, rb=rb, shuf_n=np.array(sh_n), shuf=shuf)


# ----------------------------------------------------------------------------------------
# G2: deals
# ----------------------------------------------------------------------------------------
def gen_deals():
    rs = np.random.default_rng(2024)
    seeds = np.concatenate([np.array([0, 1, 2, 3, 42, 2**31 - 2], np.int64),
                            rs.integers(0, 2**31 - 1, 506)])
    out = {}
    for P in (2, 3, 4):
        decks = np.full((len(seeds), 3, 40), -1, np.int16)
        board = np.zeros((len(seeds), 12), np.int16)
        nobles = np.full((len(seeds), 5), -1, np.int16)
        for i, s in enumerate(seeds):
            v = from_ref_state(eng.initial_state(P, int(s)))
            for t in range(3):
                decks[i, t, :len(v["decks"][t])] = v["decks"][t]
            board[i] = v["board"]
            nobles[i, :len(v["nobles"])] = v["nobles"]
        out[f"decks_p{P}"], out[f"board_p{P}"], out[f"nobles_p{P}"] = decks, board, nobles
    np.savez_compressed(os.path.join(HERE, "deals.npz"), seeds=seeds, **out)


# ----------------------------------------------------------------------------------------
# G4: env seed -> engine seed (gymnasium 0.29 seeding via numpy PCG64)
# ----------------------------------------------------------------------------------------
class SeedRecorder:
    def __init__(self):
        self.seeds = []
        self._orig = envmod.initial_state

    def __enter__(self):
        def rec(num_players=2, seed=0):
            self.seeds.append(int(seed))
            return self._orig(num_players=num_players, seed=seed)
        envmod.initial_state = rec
        return self

    def __exit__(self, *a):
        envmod.initial_state = self._orig


def gen_seeding():
    env_seeds = np.arange(1024, dtype=np.int64)
    eng_seeds = np.zeros((len(env_seeds), 5), np.int64)
    env = make_env(2)
    with SeedRecorder() as rec:
        for i, s in enumerate(env_seeds):
            rec.seeds.clear()
            env.reset(seed=int(s))
            for _ in range(4):
                env.reset()
            eng_seeds[i] = rec.seeds
    np.savez_compressed(os.path.join(HERE, "seeding.npz"), env_seeds=env_seeds, engine_seeds=eng_seeds)


# ----------------------------------------------------------------------------------------
# G3: trajectories with autoreset
# ----------------------------------------------------------------------------------------
def gen_traj(P, tables, plies, full_tables, seed_base):
    T, N = plies, tables
    action = np.zeros((N, T), np.int32)
    reward = np.zeros((N, T), np.float32)
    term = np.zeros((N, T), np.uint8)
    flags = np.zeros((N, T), np.uint8)
    to_play = np.zeros((N, T), np.int8)
    final_r = np.full((N, T, P), np.nan, np.float32)
    obs_h = np.zeros((N, T), np.uint64)
    mask_b = np.zeros((N, T), np.uint64)
    st_h = np.zeros((N, T), np.uint64)
    full_obs = np.zeros((full_tables, T, 297), np.uint8)
    reset_rows = []          # (table, ply, engine_seed, obs_digest, mask_bits, state_digest)
    reset_obs = []           # full reset obs for the first tables
    init = np.zeros((N, 4), np.uint64)  # engine_seed, obs digest, mask bits, state digest
    init_obs = np.zeros((full_tables, 297), np.uint8)
    env_seeds = np.arange(N, dtype=np.int64) + seed_base
    with SeedRecorder() as rec:
        for t in range(N):
            env = make_env(P)
            pol = np.random.default_rng(10_000 + int(env_seeds[t]))
            rec.seeds.clear()
            obs, info = env.reset(seed=int(env_seeds[t]))
            init[t] = [rec.seeds[-1], obs_digest(obs), mask_bits(info["action_mask"]),
                       digest(from_ref_state(env.state))]
            if t < full_tables:
                init_obs[t] = obs
            for k in range(T):
                m = np.asarray(info["action_mask"])
                legal = np.flatnonzero(m)
                illegal = np.flatnonzero(m == 0)
                if len(legal) == 0:
                    a = int(pol.integers(0, 45))
                elif len(illegal) and pol.random() < 0.03:
                    a = int(pol.choice(illegal))
                else:
                    a = int(pol.choice(legal))
                obs, r, te, tr, info = env.step(a)
                action[t, k], reward[t, k], term[t, k] = a, r, te
                flags[t, k] = info_flags(info)
                to_play[t, k] = info["to_play"]
                if "final_rewards" in info:
                    final_r[t, k] = [info["final_rewards"][p] for p in range(P)]
                obs_h[t, k] = obs_digest(obs)
                mask_b[t, k] = mask_bits(info["action_mask"])
                st_h[t, k] = digest(from_ref_state(env.state))
                if t < full_tables:
                    full_obs[t, k] = obs
                if te:
                    rec.seeds.clear()
                    obs, info = env.reset()
                    reset_rows.append((t, k, rec.seeds[-1], obs_digest(obs),
                                       mask_bits(info["action_mask"]), digest(from_ref_state(env.state))))
                    if t < full_tables:
                        reset_obs.append(np.asarray(obs, np.uint8))
    np.savez_compressed(
        os.path.join(HERE, f"traj_p{P}.npz"), P=P, env_seeds=env_seeds, action=action, reward=reward,
        terminated=term, flags=flags, to_play=to_play, final_rewards=final_r, obs_digest=obs_h,
        mask=mask_b, state_digest=st_h, full_obs=full_obs, init=init, init_obs=init_obs,
        reset_rows=np.array(reset_rows, np.uint64).reshape(-1, 6),
        reset_obs=np.array(reset_obs, np.uint8).reshape(-1, 297))
    return int(term.sum())


# ----------------------------------------------------------------------------------------
# G5: crafted + fuzzed states
# ----------------------------------------------------------------------------------------
def run_case(name, P, view, action):
    env = make_env(P)
    env.reset(seed=0)
    env.state = to_ref_state(view)
    before = from_ref_state(env.state)
    rec = dict(name=name, P=P, before=before, action=int(action),
               legal=mask_bits(eng.legal_moves(env.state)))
    try:
        obs, r, te, tr, info = env.step(int(action))
        rec.update(exception=None, obs=[int(x) for x in obs], reward=float(r), terminated=int(te),
                   flags=info_flags(info), mask=mask_bits(info["action_mask"]), to_play=int(info["to_play"]),
                   final_rewards=([float(info["final_rewards"][p]) for p in range(P)]
                                  if "final_rewards" in info else None),
                   after=from_ref_state(env.state))
    except (RuntimeError, ValueError) as e:
        rec.update(exception=type(e).__name__, after=from_ref_state(env.state))
    return rec


def base_view(P, seed):
    return from_ref_state(eng.initial_state(P, seed))


def first_legal(view):
    m = eng.legal_moves(to_ref_state(view))
    return next((i for i, x in enumerate(m) if x), 0)


def gen_edge_cases():
    cases = []
    # tests/test_take_reduced_colors.py:7-21 — two colours available
    v = base_view(2, 123)
    v["bank"] = [1, 0, 2, 0, 0, 0]
    cases.append(run_case("take3_two_colours", 2, v, first_legal(v)))
    # :24-36 — one colour available
    v = base_view(2, 123)
    v["bank"] = [0, 0, 0, 0, 3, 0]
    for a in (2, 9, 0):
        cases.append(run_case(f"take3_one_colour_a{a}", 2, v, a))
    # tests/test_draw_rule.py:7-24 — no legal move => draw (reserved from deck 1, revealed list empty)
    v = base_view(2, 5)
    v["bank"] = [0] * 6
    v["players"][0]["tokens"] = [10, 0, 0, 0, 0, 0]
    v["players"][0]["reserved"] = v["decks"][0][:3]
    v["players"][0]["revealed"] = [False, False, False]
    v["board"] = [-1] * 12
    for a in (0, 44, 45, -1):
        cases.append(run_case(f"no_legal_draw_a{a}", 2, v, a))
    # tests/test_rules.py:37-43 — token limit from 25 tokens (seed outside the LUT domain)
    v = base_view(2, 0)
    v["players"][0]["tokens"] = [5, 5, 5, 5, 5, 0]
    cases.append(run_case("token_limit_25", 2, v, 0))
    # tests/test_afford_nobles_obs.py:58-71 — [3,3,3,3,3,0] after reset(seed=7)
    v = base_view(2, 7)
    v["players"][0]["tokens"] = [3, 3, 3, 3, 3, 0]
    cases.append(run_case("token_return_15", 2, v, first_legal(v)))
    # gold-only overflow: non-gold exhausted first, then gold
    v = base_view(2, 11)
    v["players"][0]["tokens"] = [1, 0, 0, 0, 0, 10]
    v["bank"] = [4, 4, 4, 4, 4, 0]
    cases.append(run_case("token_return_gold", 2, v, 0))
    # tests/test_afford_nobles_obs.py:9-28 — discount + gold (card 29 costs blue 2, red 2)
    v = base_view(2, 123)
    v["players"][0]["tokens"] = [0, 1, 0, 1, 0, 1]
    v["players"][0]["bonuses"] = [0, 0, 0, 1, 0]
    v["board"][0] = 29
    v["bank"] = [4, 4, 4, 4, 4, 5]
    cases.append(run_case("buy_with_discount_and_gold", 2, v, 15))
    # :31-43 — several nobles eligible, exactly one granted (first in slot order)
    v = base_view(2, 999)
    v["players"][0]["bonuses"] = [4, 4, 4, 4, 4]
    cases.append(run_case("one_noble_per_turn", 2, v, first_legal(v)))
    # illegal action (tests/test_gym_compat.py:111-124)
    v = base_view(2, 321)
    cases.append(run_case("illegal_take2", 2, dict(v, bank=[3, 4, 4, 4, 4, 5]), 10))
    # out-of-range actions
    for a in (45, -1, 1000):
        cases.append(run_case(f"oob_{a}", 2, base_view(2, 3), a))
    # step after termination
    v = base_view(2, 4)
    v["game_over"], v["to_play"], v["winner"] = 1, 0, 1
    cases.append(run_case("step_after_terminal", 2, v, 0))
    # turn limit: move 197 -> turn_count 100 (engine/rules.py:275-279)
    v = base_view(2, 8)
    v["move_count"], v["turn_count"], v["to_play"] = 197, 99, 1
    cases.append(run_case("turn_limit", 2, v, 0))
    # turn limit overrides a prestige win at the same ply
    v = base_view(2, 9)
    v["move_count"], v["turn_count"], v["to_play"] = 197, 99, 1
    v["players"][1]["prestige"] = 14
    v["players"][1]["tokens"] = [7, 7, 7, 7, 7, 5]
    pts = [i for i, c in enumerate(v["board"]) if c >= 0 and CARDS[c].points > 0]
    cases.append(run_case("turn_limit_overrides_win", 2, v, 15 + pts[0]))
    # prestige >= 15 by player 0: game continues to player 1, then winner
    v = base_view(2, 10)
    v["players"][0]["prestige"] = 14
    v["players"][0]["tokens"] = [7, 7, 7, 7, 7, 5]
    pts = [i for i, c in enumerate(v["board"]) if c >= 0 and CARDS[c].points > 0]
    cases.append(run_case("prestige_trigger_p0", 2, v, 15 + pts[0]))
    v2 = json.loads(json.dumps(cases[-1]["after"]))
    cases.append(run_case("prestige_finish_p1", 2, v2, first_legal(v2)))
    # tie on (prestige, -cards, -reserved) -> winner None, reward 0
    v = base_view(2, 12)
    v["game_over"], v["to_play"] = 1, 1
    v["players"][0]["prestige"] = v["players"][1]["prestige"] = 15
    cases.append(run_case("tie_no_winner", 2, v, first_legal(v)))
    # tie broken by fewer cards
    v = base_view(2, 12)
    v["game_over"], v["to_play"] = 1, 1
    v["players"][0]["prestige"] = v["players"][1]["prestige"] = 15
    v["players"][0]["bonuses"] = [1, 0, 0, 0, 0]
    cases.append(run_case("tie_fewer_cards", 2, v, 0))
    # buy reserved: pop(i) shifts the later slots (engine/rules.py:253-254)
    v = base_view(2, 13)
    p = v["players"][0]
    p["reserved"], p["revealed"] = [v["decks"][0][0], 29, v["decks"][2][0]], [False, True, False]
    p["tokens"] = [0, 2, 0, 2, 0, 0]
    cases.append(run_case("buy_reserved_shift", 2, v, 43))
    # reserve blind and visible from the opponent's point of view; reserve with empty gold bank
    v = base_view(2, 14)
    v["bank"][5] = 0
    cases.append(run_case("reserve_visible_no_gold", 2, v, 27 + 5))
    v = base_view(2, 14)
    cases.append(run_case("reserve_blind_t3", 2, v, 41))
    v = base_view(2, 15)
    v["players"][1]["reserved"], v["players"][1]["revealed"] = [3, 45, 80], [True, False, True]
    cases.append(run_case("opp_hidden_reserved", 2, v, 0))
    # empty decks: refill leaves slot empty; blind reserve masked
    v = base_view(2, 16)
    v["decks"] = [[], [], []]
    v["players"][0]["tokens"] = [7, 7, 7, 7, 7, 0]
    cases.append(run_case("buy_empty_deck", 2, v, 15))
    # 4-player engine semantics: turn limit at to_play != 0 keeps going until to_play == 0
    v = base_view(4, 17)
    v["move_count"], v["turn_count"], v["to_play"] = 197, 99, 1
    cases.append(run_case("p4_turn_limit_mid_round", 4, v, first_legal(v)))
    v2 = json.loads(json.dumps(cases[-1]["after"]))
    for k in range(3):
        cases.append(run_case(f"p4_after_limit_{k}", 4, v2, first_legal(v2)))
        v2 = json.loads(json.dumps(cases[-1]["after"]))
    cases += gen_fuzz()
    with open(os.path.join(HERE, "edge_cases.json"), "w") as f:
        json.dump(cases, f, separators=(",", ":"))
    return len(cases)


def gen_fuzz(n_per_p=(400, 100, 150)):
    """Random perturbations of real mid-game states, then one env.step."""
    out = []
    rs = np.random.default_rng(77)
    for P, n in zip((2, 3, 4), n_per_p):
        env = make_env(P)
        made = 0
        game = 0
        while made < n:
            env.reset(seed=5000 + game)
            game += 1
            plies = int(rs.integers(0, 60))
            ok = True
            for _ in range(plies):
                m = eng.legal_moves(env.state)
                legal = [i for i, x in enumerate(m) if x]
                if not legal:
                    ok = False
                    break
                _, _, te, _, _ = env.step(int(rs.choice(legal)))
                if te:
                    ok = False
                    break
            if not ok:
                continue
            v = from_ref_state(env.state)
            cur = v["players"][v["to_play"]]
            kind = rs.integers(0, 6)
            if kind == 0:      # heavy tokens: exercises token return in and out of the LUT domain
                cur["tokens"] = [int(x) for x in rs.integers(0, 5, 6)]
            elif kind == 1:    # rich bonuses: nobles and discounts
                cur["bonuses"] = [int(x) for x in rs.integers(0, 6, 5)]
            elif kind == 2:    # sparse bank
                v["bank"] = [int(x) for x in rs.integers(0, 3, 6)]
            elif kind == 3:    # near the end
                cur["prestige"] = int(rs.integers(10, 16))
                cur["tokens"] = [int(x) for x in rs.integers(0, 6, 6)]
            elif kind == 4:    # late turns
                mc = int(rs.integers(180, 198)) if P == 2 else int(rs.integers(190, 202))
                v["move_count"], v["turn_count"] = mc, mc // 2 + 1
                v["to_play"] = mc % P
            else:              # random reserved cards
                k = int(rs.integers(0, 4))
                cur["reserved"] = [int(x) for x in rs.choice(90, k, replace=False)]
                cur["revealed"] = [bool(x) for x in rs.integers(0, 2, k)]
            m = eng.legal_moves(to_ref_state(v))
            legal = [i for i, x in enumerate(m) if x]
            a = int(rs.choice(legal)) if (legal and rs.random() < 0.9) else int(rs.integers(0, 45))
            out.append(run_case(f"fuzz_p{P}_{made}", P, v, a))
            made += 1
    return out


if __name__ == "__main__":
    gen_mt_kat(); print("mt_kat")
    gen_deals(); print("deals")
    gen_seeding(); print("seeding")
    print("traj p2 terminations", gen_traj(2, 256, 400, 16, 0))
    print("traj p3 terminations", gen_traj(3, 48, 200, 8, 100_000))
    print("traj p4 terminations", gen_traj(4, 96, 200, 8, 200_000))
    print("edge cases", gen_edge_cases())
