"""ctypes wrapper around the CPU oracle (oracle/splendor_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, never by the product package (splendor-gym_amd/splendor_gym).
"""
import ctypes
import json
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
LIB_PATH = os.path.join(HERE, "build", "liboracle.so")
TABLES_JSON = os.path.join(REPO, "splendor-gym_amd", "splendor_gym", "engine", "data", "tables.json")

OBS_DIM = 297
F_ILLEGAL, F_DRAW, F_TURN_LIMIT, F_AFTER_TERMINAL, F_OOB, F_RESET = 1, 2, 4, 8, 16, 32

PLAYER_DTYPE = np.dtype([("tokens", "<i4", 6), ("bonuses", "<i4", 5), ("prestige", "<i4"),
                         ("n_reserved", "<i4"), ("reserved", "<i4", 3), ("revealed", "<i4", 3),
                         ("n_nobles", "<i4"), ("nobles", "<i4", 5)])
TABLE_DTYPE = np.dtype([("num_players", "<i4"), ("bank", "<i4", 6), ("players", PLAYER_DTYPE, 4),
                        ("board", "<i4", 12), ("deck_len", "<i4", 3), ("decks", "<i4", (3, 40)),
                        ("n_nobles", "<i4"), ("nobles", "<i4", 5), ("to_play", "<i4"),
                        ("turn_count", "<i4"), ("move_count", "<i4"), ("game_over", "<i4"),
                        ("winner", "<i4"), ("turn_limit_reached", "<i4")])


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def load_tables():
    with open(TABLES_JSON) as f:
        t = json.load(f)
    return np.array(t["cards"], np.int32), np.array(t["nobles"], np.int32)


def view_to_table(v):
    r = np.zeros((), TABLE_DTYPE)
    r["num_players"] = v["P"]
    r["bank"] = v["bank"]
    for p in range(4):
        q = r["players"][p]
        q["reserved"] = -1
        q["nobles"] = -1
        if p < v["P"]:
            pv = v["players"][p]
            q["tokens"], q["bonuses"], q["prestige"] = pv["tokens"], pv["bonuses"], pv["prestige"]
            q["n_reserved"] = len(pv["reserved"])
            q["reserved"][:len(pv["reserved"])] = pv["reserved"]
            rev = list(pv["revealed"]) + [False] * (len(pv["reserved"]) - len(pv["revealed"]))
            q["revealed"][:len(pv["reserved"])] = [int(bool(x)) for x in rev[:len(pv["reserved"])]]
            q["n_nobles"] = len(pv["nobles"])
            q["nobles"][:len(pv["nobles"])] = pv["nobles"]
    r["board"] = v["board"]
    r["decks"] = -1
    for t in range(3):
        r["deck_len"][t] = len(v["decks"][t])
        r["decks"][t][:len(v["decks"][t])] = v["decks"][t]
    r["n_nobles"] = len(v["nobles"])
    r["nobles"] = -1
    r["nobles"][:len(v["nobles"])] = v["nobles"]
    for k in ("to_play", "turn_count", "move_count", "game_over", "winner", "turn_limit_reached"):
        r[k] = int(v[k])
    return r


def table_to_view(r):
    P = int(r["num_players"])
    players = []
    for p in range(P):
        q = r["players"][p]
        n = int(q["n_reserved"])
        players.append(dict(tokens=[int(x) for x in q["tokens"]], bonuses=[int(x) for x in q["bonuses"]],
                            prestige=int(q["prestige"]), reserved=[int(x) for x in q["reserved"][:n]],
                            revealed=[bool(x) for x in q["revealed"][:n]],
                            nobles=[int(x) for x in q["nobles"][:int(q["n_nobles"])]]))
    return dict(P=P, bank=[int(x) for x in r["bank"]], players=players,
                board=[int(x) for x in r["board"]],
                decks=[[int(x) for x in r["decks"][t][:int(r["deck_len"][t])]] for t in range(3)],
                nobles=[int(x) for x in r["nobles"][:int(r["n_nobles"])]],
                to_play=int(r["to_play"]), turn_count=int(r["turn_count"]),
                move_count=int(r["move_count"]), game_over=int(r["game_over"]),
                winner=int(r["winner"]), turn_limit_reached=int(r["turn_limit_reached"]))


class MT(ctypes.Structure):
    _fields_ = [("mt", ctypes.c_uint32 * 624), ("index", ctypes.c_int)]


class PCG(ctypes.Structure):
    _fields_ = [("s_hi", ctypes.c_uint64), ("s_lo", ctypes.c_uint64), ("inc_hi", ctypes.c_uint64),
                ("inc_lo", ctypes.c_uint64), ("has32", ctypes.c_uint32), ("u32", ctypes.c_uint32)]


def pcg_state_of(seed):
    """numpy PCG64 state of gymnasium 0.29's np_random after reset(seed=seed)."""
    st = np.random.PCG64(np.random.SeedSequence(seed)).state["state"]
    s, inc = st["state"], st["inc"]
    return [(s >> 64) & (2**64 - 1), s & (2**64 - 1), (inc >> 64) & (2**64 - 1), inc & (2**64 - 1)]


class Oracle:
    def __init__(self):
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        self.L = L
        P, I, U64, U32 = ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64, ctypes.c_uint32
        L.orc_set_tables.argtypes = [P, P]
        L.orc_mt_seed.argtypes = [P, U64]
        L.orc_mt_next.argtypes = [P]
        L.orc_mt_next.restype = U32
        L.orc_mt_randbelow.argtypes = [P, U32]
        L.orc_mt_randbelow.restype = U32
        L.orc_pcg_next32.argtypes = [P]
        L.orc_pcg_next32.restype = U32
        L.orc_engine_seed.argtypes = [P]
        L.orc_engine_seed.restype = ctypes.c_int64
        L.orc_initial_state.argtypes = [P, I, U32]
        L.orc_legal.argtypes = [P]
        L.orc_legal.restype = U64
        L.orc_apply.argtypes = [P, I]
        L.orc_encode.argtypes = [P, P]
        L.orc_env_step.argtypes = [P, I, P, P, P, P, P, P, P]
        L.orc_slot_size.restype = I
        L.orc_table_size.restype = I
        L.orc_vec_reset.argtypes = [P, I, I, P, P, P]
        L.orc_vec_step.argtypes = [P, I, P, P, P, P, P, P, P, P]
        L.orc_random_rollout.argtypes = [I, P, U64, ctypes.c_int64, P]
        L.orc_random_rollout.restype = ctypes.c_int64
        assert L.orc_table_size() == TABLE_DTYPE.itemsize, "spl_table_t layout mismatch"
        self.cards, self.nobles = load_tables()
        L.orc_set_tables(self.cards.ctypes.data, self.nobles.ctypes.data)

    # ---- RNG ------------------------------------------------------------------------
    def mt(self, seed):
        m = MT()
        self.L.orc_mt_seed(ctypes.byref(m), seed)
        return m

    def mt_words(self, seed, n):
        m = self.mt(seed)
        return [self.L.orc_mt_next(ctypes.byref(m)) for _ in range(n)]

    def randbelow_seq(self, seed, n, count):
        m = self.mt(seed)
        return [self.L.orc_mt_randbelow(ctypes.byref(m), n) for _ in range(count)]

    def engine_seeds(self, env_seed, count):
        p = PCG(*pcg_state_of(env_seed), 0, 0)
        return [self.L.orc_engine_seed(ctypes.byref(p)) for _ in range(count)]

    # ---- engine -----------------------------------------------------------------------
    def initial_state(self, P, seed):
        r = np.zeros((), TABLE_DTYPE)
        self.L.orc_initial_state(r.ctypes.data, P, seed)
        return table_to_view(r)

    def legal(self, view):
        r = view_to_table(view)
        return int(self.L.orc_legal(r.ctypes.data))

    def encode(self, view):
        r = view_to_table(view)
        obs = np.zeros(OBS_DIM, np.int32)
        self.L.orc_encode(r.ctypes.data, obs.ctypes.data)
        return obs

    def env_step(self, view, action):
        """One SplendorEnv.step on a copy of `view`; returns a result dict."""
        r = view_to_table(view)
        obs = np.zeros(OBS_DIM, np.int32)
        mask, rew = np.zeros(1, np.uint64), np.zeros(1, np.float32)
        term, flags, hf = np.zeros(1, np.int32), np.zeros(1, np.int32), np.zeros(1, np.int32)
        fr = np.zeros(4, np.float32)
        err = self.L.orc_env_step(r.ctypes.data, int(action), obs.ctypes.data, mask.ctypes.data,
                                  rew.ctypes.data, term.ctypes.data, flags.ctypes.data, fr.ctypes.data,
                                  hf.ctypes.data)
        out = dict(error=int(err), after=table_to_view(r))
        if not err:
            out.update(obs=obs, mask=int(mask[0]), reward=float(rew[0]), terminated=int(term[0]),
                       flags=int(flags[0]), final_rewards=(fr[:view["P"]].tolist() if hf[0] else None))
        return out


class OracleVec:
    """Batched oracle env with same-step autoreset (the semantics spl_step implements)."""

    def __init__(self, orc, n, P, env_seeds):
        self.o, self.n, self.P = orc, n, P
        self.slot_size = orc.L.orc_slot_size()
        self.buf = np.zeros(n * self.slot_size, np.uint8)
        pcg = np.array([pcg_state_of(int(s)) for s in env_seeds], np.uint64).reshape(-1)
        self.obs = np.zeros((n, OBS_DIM), np.int32)
        self.mask = np.zeros(n, np.uint64)
        orc.L.orc_vec_reset(self.buf.ctypes.data, n, P, pcg.ctypes.data, self.obs.ctypes.data,
                            self.mask.ctypes.data)

    def step(self, actions, want_final=False):
        n = self.n
        actions = np.ascontiguousarray(actions, np.int32)
        rew = np.zeros(n, np.float32)
        term, flags, win = np.zeros(n, np.uint8), np.zeros(n, np.uint8), np.zeros(n, np.int8)
        fobs = np.zeros((n, OBS_DIM), np.int32) if want_final else None
        self.o.L.orc_vec_step(self.buf.ctypes.data, n, actions.ctypes.data, self.obs.ctypes.data,
                              self.mask.ctypes.data, rew.ctypes.data, term.ctypes.data,
                              flags.ctypes.data, win.ctypes.data,
                              fobs.ctypes.data if want_final else None)
        return dict(obs=self.obs.copy(), mask=self.mask.copy(), reward=rew, terminated=term,
                    flags=flags, winner=win, final_obs=fobs)

    def table(self, i):
        raw = self.buf[i * self.slot_size:i * self.slot_size + TABLE_DTYPE.itemsize]
        return table_to_view(np.frombuffer(raw.tobytes(), TABLE_DTYPE)[0])


def mask_bits_to_int8(bits):
    bits = np.asarray(bits, np.uint64)
    return ((bits[..., None] >> np.arange(45, dtype=np.uint64)) & np.uint64(1)).astype(np.int8)
