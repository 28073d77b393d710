"""CPU-only tests: C-ABI exports, host-side seeding/layout logic, the device RNG formulation
compiled for the host, and the gloo multi-process sharding path."""
import ctypes
import json
import os
import re
import subprocess
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INCLUDE = os.path.join(REPO, "include")


def header_functions():
    names = set()
    for h in os.listdir(INCLUDE):
        src = open(os.path.join(INCLUDE, h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        names |= set(re.findall(r"^\s*(?:const\s+)?(?:volatile\s+)?[a-z_0-9]+\s*\*?\s*(spl_[a-z_0-9]+)\s*\(", src, flags=re.M))
    return names


def test_library_exports_every_header_symbol():
    from splendor_gym import _native
    lib = _native.load_library()  # dlopen only: no GPU needed
    declared = header_functions()
    assert len(declared) >= 15, declared
    assert declared == set(_native.SIGNATURES), declared ^ set(_native.SIGNATURES)
    for name in declared:
        assert hasattr(lib, name), name
    assert lib.spl_abi_version() == _native.ABI_VERSION == 9


def test_abi_host_side_errors():
    """Argument errors are reported before any device work (runs without a GPU)."""
    from splendor_gym import _native
    lib = _native.load_library()
    out = ctypes.c_void_p()
    assert lib.spl_ctx_create(0, None, None, ctypes.byref(out)) == -1
    assert b"null" in lib.spl_last_error()
    assert lib.spl_arena_bytes(0, 2) == -1 and lib.spl_arena_bytes(10, 5) == -1
    arena = _native.ArenaDesc(None, 0, 10, 2, 0, 0)
    assert lib.spl_step(None, ctypes.byref(arena), None, None) == -1


def test_policy_abi_host_side_errors():
    """spl_policy_* argument checks (include/splendor_policy.h) run before any device work."""
    from splendor_gym import _native
    lib = _native.load_library()
    # bf16: actor 18 chunks, full image 35 chunks + the fp32 critic output layer; fp32: 35 / 67 chunks + tail
    assert lib.spl_policy_bytes(0, 1) == 18 * 20480 and lib.spl_policy_bytes(1, 1) == 35 * 20480 + 272 * 4
    # fp32 images (spl_policy32.hip): exact (SPL_PREC_FP32, 0) 31-KB chunks of three bf16 planes of a
    # 16-row tile + its biases and row factors; two fp16 planes (SPL_PREC_FP32_F16X2, 2) 21-KB chunks
    assert lib.spl_policy_bytes(0, 0) == 35 * 31744 and lib.spl_policy_bytes(1, 0) == 67 * 31744 + 272 * 4
    assert lib.spl_policy_bytes(0, 2) == 35 * 21504 and lib.spl_policy_bytes(1, 2) == 67 * 21504 + 272 * 4
    assert lib.spl_policy_bytes(0, 9) == -1 and lib.spl_policy_bytes(0, 3) == -1
    assert lib.spl_policy_pack(None, None, 0, None, None) == -1
    assert b"actor" in lib.spl_last_error()
    assert lib.spl_policy_act(None, 0, 1, None, None) == -1
    args = _native.ActArgs(obs=256, mask=256, action=256, mode=0, image=0)
    args.obs = 258  # misaligned observations
    assert lib.spl_policy_act(ctypes.c_void_p(4096), lib.spl_policy_bytes(0, 0), 1, ctypes.byref(args), None) == -1
    assert b"obs" in lib.spl_last_error()
    args.obs, args.value = 256, 256  # critic requested from an actor-only image
    assert lib.spl_policy_act(ctypes.c_void_p(4096), lib.spl_policy_bytes(0, 0), 1, ctypes.byref(args), None) == -1
    assert b"critic" in lib.spl_last_error() or b"value" in lib.spl_last_error()
    # an image size that does not match args->image (a full image passed as actor-only, or the
    # reverse) is refused instead of evaluating the wrong chunks
    args.value = None
    for image, size in ((0, lib.spl_policy_bytes(1, 0)), (1, lib.spl_policy_bytes(0, 0)),
                        (2, lib.spl_policy_bytes(0, 0)), (0, lib.spl_policy_bytes(0, 1)), (3, 35 * 20480),
                        (4, lib.spl_policy_bytes(0, 0)), (0, lib.spl_policy_bytes(0, 2))):
        args.image = image
        assert lib.spl_policy_act(ctypes.c_void_p(4096), size, 1, ctypes.byref(args), None) == -1
        assert b"packed_bytes" in lib.spl_last_error()
    args.image = 0
    args.value, args.mode = None, 7
    assert lib.spl_policy_act(ctypes.c_void_p(4096), lib.spl_policy_bytes(0, 0), 1, ctypes.byref(args), None) == -1
    # compact rows (policy ABI 3): exclusive with obs, fp32 images only, 4-byte aligned
    args.mode, args.obs_u8 = 1, 512
    assert lib.spl_policy_act(ctypes.c_void_p(4096), lib.spl_policy_bytes(0, 0), 1, ctypes.byref(args), None) == -1
    assert b"exclusive" in lib.spl_last_error()
    args.obs, args.image = None, 2  # bf16 image
    assert lib.spl_policy_act(ctypes.c_void_p(4096), lib.spl_policy_bytes(0, 1), 1, ctypes.byref(args), None) == -1
    assert b"fp32" in lib.spl_last_error()
    args.image, args.obs_u8 = 0, 514
    assert lib.spl_policy_act(ctypes.c_void_p(4096), lib.spl_policy_bytes(0, 0), 1, ctypes.byref(args), None) == -1
    assert b"aligned" in lib.spl_last_error()


def test_dual_abi_host_side_errors():
    """spl_dual_* argument checks (include/splendor_dual.h) run before any launch."""
    from splendor_gym import _native
    lib = _native.load_library()
    io = _native.DualIo()
    assert lib.spl_dual_finish(0, ctypes.byref(io), None) == -1
    assert lib.spl_dual_finish(8, ctypes.byref(io), None) == -1 and b"null" in lib.spl_last_error()
    assert lib.spl_dual_finish_draw(8, ctypes.byref(io), None, None) == -1 and b"draw" in lib.spl_last_error()
    d = _native.DualDraw(episode=256, group_of=256, pool_len=3, p_current=0.25)  # pool slots missing
    assert lib.spl_dual_finish_draw(8, ctypes.byref(io), ctypes.byref(d), None) == -1
    d.pool_slots, d.p_current = 256, 1.5
    assert lib.spl_dual_finish_draw(8, ctypes.byref(io), ctypes.byref(d), None) == -1
    assert b"p_current" in lib.spl_last_error()


def test_arena_layout_sizes():
    from splendor_gym import _native
    lib = _native.load_library()
    for n in (1, 63, 64, 65536):
        for P in (2, 3, 4):
            words = 9 + 4 * P
            b = int(lib.spl_arena_bytes(n, P))
            # state planes + 5 pool planes + 4 deck slot records x 128 B + 64 B PCG record, then per pair
            # of 64-table workgroups 24 staged steps (64 tables x 25 state words) and 50 flag lines
            # (rollout-store delegation), then the legal-mask cache (2 u32 planes, ABI 9)
            deleg = (n // 128) * (24 * 64 * 25 * 4 + 50 * 128)
            assert b >= (words + 5) * 4 * n + 512 * n + 64 * n + deleg + 8 * n
            assert b % 256 == 0 and b <= (words + 5) * 4 * n + 584 * n + deleg + 7 * 256


def test_table_dtype_matches_oracle_struct():
    from oracle.oracle import Oracle, TABLE_DTYPE as ORC
    from splendor_gym._native import TABLE_DTYPE
    assert TABLE_DTYPE == ORC
    assert TABLE_DTYPE.itemsize == Oracle().L.orc_table_size()


def test_seeding_matches_numpy_generator():
    from splendor_gym.seeding import pcg64_state, vector_seeds
    for seed in (0, 1, 12345, 2**40):
        s = pcg64_state(seed)
        st = np.random.PCG64(np.random.SeedSequence(seed)).state["state"]
        assert (s[0] << 64 | s[1]) == st["state"] and (s[2] << 64 | s[3]) == st["inc"]
    assert vector_seeds(5, 3) == [5, 6, 7]
    assert vector_seeds(None, 3) is None
    with pytest.raises(ValueError):
        vector_seeds([1, 2], 3)


def test_engine_seed_stream_matches_gymnasium_semantics():
    """The device continues numpy's PCG64 stream for engine seeds; the oracle restatement of
    that continuation equals numpy's own Generator.integers(0, 2**31-1)."""
    from oracle.oracle import Oracle
    o = Oracle()
    for seed in (0, 3, 99, 2024):
        g = np.random.Generator(np.random.PCG64(np.random.SeedSequence(seed)))
        assert o.engine_seeds(seed, 6) == [int(g.integers(0, 2**31 - 1)) for _ in range(6)]


def test_constants_match_reference_layout():
    from splendor_gym.engine import encode as E
    assert (E.TAKE3_OFFSET, E.TAKE2_OFFSET, E.BUY_VISIBLE_OFFSET, E.RESERVE_VISIBLE_OFFSET,
            E.RESERVE_BLIND_OFFSET, E.BUY_RESERVED_OFFSET, E.TOTAL_ACTIONS) == (0, 10, 15, 27, 39, 42, 45)
    assert E.OBSERVATION_DIM == 297
    assert E.TAKE3_COMBOS[0] == (0, 1, 2) and E.TAKE3_COMBOS[-1] == (2, 3, 4)
    assert E.encode_buy_visible_index(2, 3) == 22 and E.encode_reserve_blind_index(3) == 41


def test_host_state_record_roundtrip():
    from oracle.oracle import Oracle, view_to_table
    from splendor_gym.engine.state import SplendorState
    from splendor_gym.scripts.game_logger import format_game_state
    o = Oracle()
    v = o.initial_state(2, 42)
    rec = view_to_table(v)
    s = SplendorState.from_record(rec)
    assert s.to_record().tobytes() == rec.tobytes()
    assert s.board[1][0].id == v["board"][0] and s.bank == [4, 4, 4, 4, 4, 5]
    assert "Bank" in format_game_state(s)


def test_device_mt_stream_formulation_on_host(tmp_path):
    """The register-only MT19937 stream of csrc/spl_rng.h, compiled for the host, equals the
    oracle's full-state MT19937 for 454 outputs (1- and 2-word keys)."""
    exe = tmp_path / "mtstream"
    orc = tmp_path / "orc.o"
    subprocess.run(["gcc", "-O2", "-c", "-o", str(orc), os.path.join(REPO, "oracle", "splendor_oracle.c")], check=True)
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", str(exe), os.path.join(REPO, "tests", "native", "mtstream_host.cpp"),
                    str(orc)], check=True)
    r = subprocess.run([str(exe), "400"], capture_output=True, text=True)
    assert r.returncode == 0 and "OK" in r.stdout, r.stdout + r.stderr


def test_shard_ranges():
    from splendor_gym.parallel import shard_range
    for n, w in ((65536, 8), (1000, 3), (5, 4)):
        rs = [shard_range(n, r, w) for r in range(w)]
        assert rs[0][0] == 0 and rs[-1][1] == n
        assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
        assert max(b - a for a, b in rs) - min(b - a for a, b in rs) <= 1


def _gloo_worker(rank, world, port, q):
    import torch
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    from splendor_gym.parallel import gather_returns, init_distributed, max_over_ranks, shard_range
    init_distributed(backend="gloo")
    n_global = 1001
    lo, hi = shard_range(n_global, rank, world)
    ids = torch.arange(lo, hi, dtype=torch.float32)
    ret, cnt = gather_returns(ids * 0.5, (ids % 7).to(torch.int64), n_global=n_global)
    t = max_over_ranks(float(rank) + 0.25)
    q.put((rank, ret.tolist(), cnt.tolist(), t))
    import torch.distributed as dist
    dist.destroy_process_group()


def test_gloo_two_ranks_gather_returns():
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29600 + os.getpid() % 300
    procs = [ctx.Process(target=_gloo_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ret, cnt, t in res:
        assert ret == [i * 0.5 for i in range(1001)]
        assert cnt == [i % 7 for i in range(1001)]
        assert t == 1.25


def _census_worker(rank, world, port, same, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    sys.path.insert(0, REPO)
    import bench
    from splendor_gym.parallel import device_census, init_distributed
    init_distributed(backend="gloo")
    census = device_census("hostA/pci 0000:05:00" if same else f"hostA/pci 0000:0{rank + 5}:00")
    rec = bench.node_fields(census, "env-steps/sec (whole node), 2p 65536 tables/GPU")
    q.put((rank, census, rec))
    import torch.distributed as dist
    dist.destroy_process_group()


@pytest.mark.parametrize("same", [True, False])
def test_gloo_device_census_flags_shared_devices(same):
    """two ranks on ONE card (the one-GPU rehearsal) report n_gpus 1, ranks 2,
    shared_device true and a metric that is not a whole-node figure; two ranks on two cards report 2."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29400 + os.getpid() % 150 + (150 if same else 0)
    procs = [ctx.Process(target=_census_worker, args=(r, 2, port, same, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, census, rec in res:
        assert census["ranks"] == 2 and census["shared_device"] is same
        assert rec["n_gpus"] == (1 if same else 2) and rec["ranks"] == 2 and rec["shared_device"] is same
        assert ("whole node" in rec["metric"]) is (not same)
        assert len(rec["devices"]) == 2


_LAUNCHED_RANK = r'''
import json, os, sys
sys.path[:0] = [sys.argv[1], os.path.join(sys.argv[1], "splendor-gym_amd")]
import torch
from splendor_gym.parallel import (device_census, gather_returns, init_distributed, max_over_ranks,
                                   require_distinct_devices, shard_range)
rank, world, local = init_distributed(backend="gloo")
same = sys.argv[3] == "same"
census = device_census("hostA/pci 0000:05:00" if same else f"hostA/pci 0000:0{local + 5}:00")
err = require_distinct_devices(census, world)
if err is not None:
    print(err, file=sys.stderr)
    sys.exit(3)
lo, hi = shard_range(1001, rank, world)
ids = torch.arange(lo, hi, dtype=torch.float32)
ret, cnt = gather_returns(ids * 0.5, (ids % 7).to(torch.int64), n_global=1001)
t = max_over_ranks(float(rank) + 0.25)
with open(os.path.join(sys.argv[2], f"rank{rank}.json"), "w") as f:
    json.dump({"rank": rank, "world": world, "local": local, "env": os.environ["SPLENDOR_SELF_LAUNCHED"],
               "census": census, "ret_ok": ret.tolist() == [i * 0.5 for i in range(1001)],
               "cnt_ok": cnt.tolist() == [i % 7 for i in range(1001)], "max": t}, f)
'''


@pytest.mark.parametrize("world", [2, 4])
def test_self_launched_ranks_over_gloo(tmp_path, world):
    """bench.py --gpus N without a launcher starts N ranks itself
    (parallel.launch_local_ranks).  Two and four ranks over gloo on CPU (1 001 tables: shards of
    unequal size at four): each gets its rank / local rank / world and the rendezvous, the census sees
    one device per rank, gather_returns and max_over_ranks agree."""
    from splendor_gym.parallel import launch_local_ranks
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    rc = launch_local_ranks(world, [sys.executable, "-c", _LAUNCHED_RANK, REPO, str(tmp_path), "distinct"], env=env)
    assert rc == 0
    recs = [json.load(open(tmp_path / f"rank{r}.json")) for r in range(world)]
    for r, rec in enumerate(recs):
        assert rec["rank"] == r and rec["local"] == r and rec["world"] == world and rec["env"] == "1"
        assert rec["census"]["devices"] == world and not rec["census"]["shared_device"]
        assert rec["ret_ok"] and rec["cnt_ok"] and rec["max"] == world - 1 + 0.25


def test_self_launched_ranks_on_one_device_fail(tmp_path):
    """Self-launched ranks that land on ONE device exit non-zero (no N-GPU figure from a shared card)."""
    from splendor_gym.parallel import launch_local_ranks
    rc = launch_local_ranks(2, [sys.executable, "-c", _LAUNCHED_RANK, REPO, str(tmp_path), "same"])
    assert rc == 3
    assert not list(tmp_path.glob("rank*.json"))


def test_self_launched_rehearsal_on_one_device_is_labelled(tmp_path):
    """SPLENDOR_SHARED_DEVICE_REHEARSAL=1: self-launched ranks on one device run (gloo) and are reported as
    a shared-device rehearsal (bench.node_fields), not refused."""
    from splendor_gym.parallel import launch_local_ranks
    env = dict(os.environ, SPLENDOR_SHARED_DEVICE_REHEARSAL="1")
    rc = launch_local_ranks(2, [sys.executable, "-c", _LAUNCHED_RANK, REPO, str(tmp_path), "same"], env=env)
    assert rc == 0
    sys.path.insert(0, REPO)
    import bench
    for r in range(2):
        rec = json.load(open(tmp_path / f"rank{r}.json"))
        assert rec["census"]["shared_device"] and rec["census"]["devices"] == 1
        line = bench.node_fields(rec["census"], "env-steps/sec (whole node), 2p 65536 tables/GPU")
        assert "shared-device rehearsal" in line["metric"] and line["n_gpus"] == 1 and line["ranks"] == 2


def test_launcher_stops_the_other_ranks_when_one_fails():
    """A failing rank ends the launch with its status and the others are terminated (none is left
    waiting in a collective)."""
    import time
    from splendor_gym.parallel import launch_local_ranks
    code = "import os, sys, time\nif os.environ['RANK'] == '1': sys.exit(5)\ntime.sleep(120)\n"
    t = time.perf_counter()
    rc = launch_local_ranks(2, [sys.executable, "-c", code])
    assert rc == 5 and time.perf_counter() - t < 60


def test_bench_gpus_n_refuses_fewer_devices(capsys):
    """`python bench.py --gpus 2` on a node with one GPU exits 2 with a device-count message and runs
    nothing; at --gpus 1 bench.main never enters the launcher."""
    sys.path.insert(0, REPO)
    import bench
    assert bench.self_launch(2, ["--gpus", "2"], device_count=1) == 2
    assert "shows 1 GPU(s); a run on 2 GPUs needs 2" in capsys.readouterr().err
    assert bench.self_launch(8, ["--gpus", "8"], device_count=0) == 2


def test_single_hip_runtime_after_load():
    """The engine library must share torch's HIP runtime (one libamdhip64 in the process)."""
    import re
    import subprocess
    import sys
    code = ("import sys; sys.path.insert(0, %r); from splendor_gym import _native; _native.load_library(); "
            "import re; m = open('/proc/self/maps').read(); "
            "print(len(set(re.findall(r'\\S*libamdhip64\\S*', m))))") % os.path.join(REPO, "splendor-gym_amd")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip().splitlines()[-1] == "1"


def test_fresh_deal_mask_constant():
    """k_step's autoreset mask is the constant kFreshDealMask (spl_engine.hip): legal_moves of
    every fresh deal, checked here on the oracle over many deals and player counts."""
    import re
    from oracle.oracle import Oracle
    src = open(os.path.join(REPO, "splendor-gym_amd", "csrc", "spl_engine.hip")).read()
    assert re.search(r"kFreshDealMask = \(\(1ull << 15\) - 1ull\) \| \(\(\(1ull << 15\) - 1ull\) << 27\)", src)
    want = ((1 << 15) - 1) | (((1 << 15) - 1) << 27)
    o = Oracle()
    for P in (2, 3, 4):
        for s in range(0, 200000, 1999):
            assert o.legal(o.initial_state(P, s)) == want, (P, s)


def test_oracle_under_address_and_undefined_sanitizers(tmp_path):
    """the CPU restatement under ASan + UBSan (gcc -fsanitize=address,undefined,
    no recovery): deals, long random rollouts and crafted extreme steps (tests/native/oracle_sanitize.c)."""
    import numpy as np
    from oracle.oracle import load_tables
    cards, nobles = load_tables()
    tables = tmp_path / "tables.bin"
    tables.write_bytes(np.concatenate([cards.reshape(-1), nobles.reshape(-1)]).astype(np.int32).tobytes())
    exe = tmp_path / "oracle_san"
    subprocess.run(["gcc", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                    "-fno-omit-frame-pointer", "-o", str(exe), os.path.join(REPO, "tests", "native", "oracle_sanitize.c"),
                    os.path.join(REPO, "oracle", "splendor_oracle.c")], check=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    env.pop("LD_PRELOAD", None)
    r = subprocess.run([str(exe), str(tables)], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0 and r.stdout.startswith("OK"), r.stdout[-2000:] + r.stderr[-4000:]


def test_bounds_check_hook_absent_from_product_build():
    import ctypes
    from splendor_gym import _native
    lib = _native.load_library()
    v = ctypes.c_uint32()
    assert lib.spl_debug_bounds_flags(ctypes.byref(v), 0) == -1  # product library: not a checked build
    assert b"bounds-check" in lib.spl_last_error()
    assert lib.spl_debug_set_stream_limit(0) == -1 and lib.spl_debug_set_stream_limit(455) == -1


def test_edited_cards_make_a_card_table():
    """Host views own their Card objects (the reference loads fresh cards per game): an in-place cost
    edit (tests/test_afford_nobles_obs.py:16-17) shows as that state's device card table, a derived
    state keeps the edited object, and the canonical cards stay untouched."""
    from oracle.oracle import Oracle, view_to_table
    from splendor_gym.engine.state import SplendorState, canonical_card_rows, cards_by_id
    rec = view_to_table(Oracle().initial_state(2, 123))
    s = SplendorState.from_record(rec)
    assert s.card_table() is None
    card = s.board[1][0]
    card.cost = {"red": 2, "blue": 2}
    tbl = s.card_table()
    base = canonical_card_rows()
    assert tbl.shape == (90, 8) and tbl.dtype == np.int32
    assert tbl[card.id].tolist() == [card.tier, ["white", "blue", "green", "red", "black"].index(card.color),
                                     card.points, 0, 2, 0, 2, 0]
    assert np.array_equal(np.delete(tbl, card.id, 0), np.delete(base, card.id, 0))
    derived = SplendorState.from_record(rec, cards=s.cards())
    assert derived.board[1][0] is card and np.array_equal(derived.card_table(), tbl)
    assert dict(cards_by_id()[card.id].cost) != card.cost
    fresh = SplendorState.from_record(rec)
    assert fresh.board[1][0] is not card and fresh.card_table() is None


def test_launcher_stops_its_ranks_on_sigterm(tmp_path):
    """SIGTERM to the launching process (a driver's time limit) ends its ranks too: none is orphaned."""
    import signal
    import subprocess
    import time
    pids = tmp_path / "pids"
    pids.mkdir()
    rank = ("import os, sys, time\nopen(os.path.join(sys.argv[1], os.environ['RANK']), 'w').write(str(os.getpid()))\n"
            "time.sleep(120)\n")
    parent = ("import sys\nsys.path[:0] = [sys.argv[1]]\nfrom splendor_gym.parallel import launch_local_ranks\n"
              "sys.exit(launch_local_ranks(2, [sys.executable, '-c', sys.argv[2], sys.argv[3]]))\n")
    p = subprocess.Popen([sys.executable, "-c", parent, os.path.join(REPO, "splendor-gym_amd"), rank, str(pids)])
    t = time.perf_counter()
    while len(list(pids.iterdir())) < 2 and time.perf_counter() - t < 240:  # the parent imports torch first
        time.sleep(0.1)
    children = [int(f.read_text()) for f in pids.iterdir()]
    assert len(children) == 2
    p.send_signal(signal.SIGTERM)
    assert p.wait(timeout=60) == 128 + signal.SIGTERM
    for pid in children:
        try:
            os.kill(pid, 0)
            alive = True
        except ProcessLookupError:
            alive = False
        assert not alive, pid
