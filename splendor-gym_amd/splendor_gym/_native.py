"""ctypes binding of the HIP engine's C-ABI (include/splendor_amd.h).

The shared library ``libsplendor_amd.so`` is built in-tree by ``__graft_entry__.build()`` (or
``make -C splendor-gym_amd/csrc``).  There is no CPU fallback: if the library or a HIP device
is missing, :func:`load` raises, and every env constructor that needs it fails loudly.
"""
import ctypes
import os

import numpy as np

LIB_NAME = "libsplendor_amd.so"
ABI_VERSION = 9

# per-table flag bits (include/splendor_amd.h)
POLICY_UNIFORM, POLICY_GREEDY_V1, POLICY_BASIC_PRIORITY = 0, 1, 2  # SPL_POLICY_* (device next_actions)
F_ILLEGAL, F_DRAW, F_TURN_LIMIT = 0x01, 0x02, 0x04
F_AFTER_TERMINAL, F_OOB, F_RESET, F_RNG_LIMIT = 0x08, 0x10, 0x20, 0x40
F_FAULT = 0x80  # SPL_F_FAULT: the launch faulted (spl_ctx_faults), this step was not written

OBS_DIM = 297
OBS_U8 = 300  # spl_step_args_t.obs_u8 row: the 297 observation bytes, move_count >> 8, two zero bytes
NUM_ACTIONS = 45

c_void_p, c_int32, c_int64, c_uint64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64


class ArenaDesc(ctypes.Structure):
    """spl_arena_t"""
    _fields_ = [("base", c_void_p), ("bytes", c_int64), ("n", c_int32), ("players", c_int32),
                ("steps", c_int64), ("epoch", c_int64)]


class StepArgs(ctypes.Structure):
    """spl_step_args_t"""
    _fields_ = [("actions", c_void_p), ("obs", c_void_p), ("mask", c_void_p), ("reward", c_void_p),
                ("terminated", c_void_p), ("flags", c_void_p), ("winner", c_void_p),
                ("final_obs", c_void_p), ("autoreset", c_int32), ("policy", c_int32), ("next_actions", c_void_p),
                ("ply_base", c_void_p), ("policy_seed", c_uint64), ("ply", c_uint64), ("table0", c_int64),
                ("ep_return", c_void_p), ("ep_count", c_void_p), ("info", c_void_p), ("errors", c_void_p),
                ("obs_u8", c_void_p), ("gate_terminated", c_void_p), ("gate_flags", c_void_p)]


class MlpDesc(ctypes.Structure):
    """spl_mlp_t (include/splendor_policy.h)"""
    _fields_ = [("w1", c_void_p), ("b1", c_void_p), ("w2", c_void_p), ("b2", c_void_p), ("w3", c_void_p),
                ("b3", c_void_p)]


class ActArgs(ctypes.Structure):
    """spl_act_args_t (include/splendor_policy.h)"""
    _fields_ = [("obs", c_void_p), ("mask", c_void_p), ("action", c_void_p), ("logprob", c_void_p),
                ("entropy", c_void_p), ("value", c_void_p), ("logits", c_void_p), ("seed", c_uint64),
                ("ply", c_uint64), ("ply_base", c_void_p), ("table0", c_int64), ("mode", c_int32), ("image", c_int32),
                ("obs_u8", c_void_p)]


ACT_SAMPLE, ACT_GREEDY, ACT_VALUE = 0, 1, 2  # SPL_ACT_*
PREC_FP32, PREC_BF16, PREC_FP32_F16X2 = 0, 1, 2    # SPL_PREC_* (FP32: exact three bf16 planes)
IMG_CRITIC = 1                 # SPL_IMG_CRITIC


class DualIo(ctypes.Structure):
    """spl_dual_io_t (include/splendor_dual.h)"""
    _fields_ = [(k, c_void_p) for k in ("reward_a", "reward_b", "terminated_a", "terminated_b", "flags_a", "flags_b",
                                        "winner_a", "winner_b", "agent_reward", "opp_reward", "done",
                                        "game_ended_on", "info_flags", "obs", "final_obs", "opp_obs",
                                        "step_counter")]


class DualDraw(ctypes.Structure):
    """spl_dual_draw_t (include/splendor_dual.h)"""
    _fields_ = [("episode", c_void_p), ("group_of", c_void_p), ("group_prev", c_void_p), ("pool_slots", c_void_p),
                ("pool_len", c_int32), ("p_current", ctypes.c_float), ("seed", c_uint64), ("table0", c_int64)]


DUAL_ILLEGAL, DUAL_DRAW, DUAL_TURN_LIMIT = 0x01, 0x02, 0x04  # SPL_DUAL_*


# spl_table_t (include/splendor_table.h) as a numpy structured dtype
PLAYER_DTYPE = np.dtype([("tokens", "<i4", 6), ("bonuses", "<i4", 5), ("prestige", "<i4"),
                         ("n_reserved", "<i4"), ("reserved", "<i4", 3), ("revealed", "<i4", 3),
                         ("n_nobles", "<i4"), ("nobles", "<i4", 5)])
TABLE_DTYPE = np.dtype([("num_players", "<i4"), ("bank", "<i4", 6), ("players", PLAYER_DTYPE, 4),
                        ("board", "<i4", 12), ("deck_len", "<i4", 3), ("decks", "<i4", (3, 40)),
                        ("n_nobles", "<i4"), ("nobles", "<i4", 5), ("to_play", "<i4"),
                        ("turn_count", "<i4"), ("move_count", "<i4"), ("game_over", "<i4"),
                        ("winner", "<i4"), ("turn_limit_reached", "<i4")])

# every symbol the header declares (tests/test_host_cpu.py::test_library_exports_every_header_symbol
# checks that the library exports them)
SIGNATURES = {
    "spl_abi_version": ([], c_int32),
    "spl_last_error": ([], ctypes.c_char_p),
    "spl_ctx_create": ([c_int32, c_void_p, c_void_p, ctypes.POINTER(c_void_p)], c_int32),
    "spl_ctx_destroy": ([c_void_p], c_int32),
    "spl_ctx_set_refill_period": ([c_void_p, c_int32], c_int32),
    "spl_ctx_set_refill_fused": ([c_void_p, c_int32], c_int32),
    "spl_ctx_set_rollout_pipeline": ([c_void_p, c_int32], c_int32),
    "spl_ctx_set_rollout_delegation": ([c_void_p, c_int32], c_int32),
    "spl_ctx_set_partner_lead": ([c_void_p, c_int32], c_int32),
    "spl_ctx_set_step_tail": ([c_void_p, c_int32], c_int32),
    "spl_ctx_token_lut": ([c_void_p, c_void_p, c_int64], c_int64),
    "spl_ctx_faults": ([c_void_p, ctypes.POINTER(c_uint64), c_int32], c_int32),
    "spl_ctx_fault_word": ([c_void_p], c_void_p),
    "spl_ctx_launches": ([c_void_p], c_uint64),
    "spl_host_mapped": ([c_void_p, ctypes.POINTER(c_int32)], c_int32),
    "spl_debug_set_spin_limit": ([c_int64], c_int32),
    "spl_debug_partner_stats": ([c_void_p, c_int32], c_int32),
    "spl_rollout_kernel_name": ([c_void_p, c_int32, c_int32, c_int32], ctypes.c_char_p),
    "spl_arena_bytes": ([c_int32, c_int32], c_int64),
    "spl_arena_init": ([c_void_p, ctypes.POINTER(ArenaDesc), c_void_p], c_int32),
    "spl_reset": ([c_void_p, ctypes.POINTER(ArenaDesc), c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
                  c_int32),
    "spl_debug_set_stream_limit": ([c_int32], c_int32),
    "spl_debug_bounds_flags": ([c_void_p, c_int32], c_int32),
    "spl_deal": ([c_void_p, ctypes.POINTER(ArenaDesc), c_void_p, c_void_p, c_void_p, c_void_p, c_void_p], c_int32),
    "spl_step": ([c_void_p, ctypes.POINTER(ArenaDesc), ctypes.POINTER(StepArgs), c_void_p], c_int32),
    "spl_rollout": ([c_void_p, ctypes.POINTER(ArenaDesc), ctypes.POINTER(StepArgs), c_int32, c_int32, c_void_p],
                    c_int32),
    "spl_refill": ([c_void_p, ctypes.POINTER(ArenaDesc), c_void_p], c_int32),
    "spl_encode": ([c_void_p, ctypes.POINTER(ArenaDesc), c_void_p, c_void_p], c_int32),
    "spl_legal": ([c_void_p, ctypes.POINTER(ArenaDesc), c_void_p, c_void_p], c_int32),
    "spl_step_info": ([c_int32, c_void_p, c_void_p, c_void_p, c_void_p], c_int32),
    "spl_sample_uniform": ([c_void_p, c_int32, c_void_p, c_void_p, c_uint64, c_uint64, c_int64, c_void_p],
                           c_int32),
    "spl_table_download": ([c_void_p, ctypes.POINTER(ArenaDesc), c_int32, c_int32, c_void_p, c_void_p],
                           c_int32),
    "spl_table_upload": ([c_void_p, ctypes.POINTER(ArenaDesc), c_int32, c_int32, c_void_p, c_void_p],
                         c_int32),
    # include/splendor_policy.h
    "spl_policy_bytes": ([c_int32, c_int32], c_int64),
    "spl_policy_pack": ([ctypes.POINTER(MlpDesc), ctypes.POINTER(MlpDesc), c_int32, c_void_p, c_void_p], c_int32),
    "spl_policy_act": ([c_void_p, c_int64, c_int32, ctypes.POINTER(ActArgs), c_void_p], c_int32),
    # include/splendor_dual.h
    "spl_dual_gate": ([c_int32, c_void_p, c_void_p, c_void_p, c_void_p], c_int32),
    "spl_dual_finish": ([c_int32, ctypes.POINTER(DualIo), c_void_p], c_int32),
    "spl_dual_finish_draw": ([c_int32, ctypes.POINTER(DualIo), ctypes.POINTER(DualDraw), c_void_p], c_int32),
    "spl_dual_draw_opponents": ([c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_int32, ctypes.c_float, c_uint64,
                                 c_int64, c_void_p], c_int32),
    "spl_policy_group_scratch_bytes": ([c_int32, c_int32], c_int64),
    "spl_policy_act_grouped": ([c_void_p, c_int64, c_int32, c_void_p, c_void_p, c_int32, ctypes.POINTER(ActArgs),
                                c_void_p], c_int32),
}


class NativeError(RuntimeError):
    pass


def lib_path():
    return os.environ.get("SPLENDOR_AMD_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), LIB_NAME)


_LIB = None


def load_library():
    """dlopen the engine library and declare its signatures (no device is touched)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    # torch bundles its own HIP runtime (SONAME libamdhip64.so.7).  Load it FIRST so this
    # library binds to the same runtime; dlopen-ing ours first would pull /opt/rocm's runtime
    # in beside torch's and leave one of them without devices.
    import torch  # noqa: F401
    path = lib_path()
    if not os.path.exists(path):
        raise ImportError(f"splendor_gym: HIP engine library not found at {path}; build it with "
                          "`python -c 'import __graft_entry__ as g; g.build()'` (no CPU fallback exists)")
    lib = ctypes.CDLL(path)
    for name, (argtypes, restype) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.argtypes = argtypes
        fn.restype = restype
    if lib.spl_abi_version() != ABI_VERSION:
        raise ImportError(f"splendor_gym: ABI version {lib.spl_abi_version()} != {ABI_VERSION}")
    _LIB = lib
    return lib


def check(lib, code):
    if code < 0:
        raise NativeError(f"splendor engine error {code}: {lib.spl_last_error().decode()}")
    return code


class LaunchFault(RuntimeError):
    """A launch lost an internal hand-off (include/splendor_amd.h spl_ctx_faults): its outputs from
    the faulted step on are not written (SPL_F_FAULT) and the tables must be reset."""


def require_gpu():
    import torch
    if not torch.cuda.is_available():
        raise RuntimeError("splendor_gym: the HIP engine needs a ROCm GPU (torch.cuda.is_available() is False); "
                           "there is no CPU fallback")
    return torch


def ptr(t):
    """Raw device pointer of a torch tensor (None -> NULL)."""
    return None if t is None else c_void_p(t.data_ptr())
