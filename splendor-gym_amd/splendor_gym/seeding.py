"""gymnasium-0.29-compatible seeding, reduced to what the device needs.

The reference env draws each episode's engine seed from its gymnasium ``np_random``
(envs/splendor_env.py:42-43): ``Generator(PCG64(SeedSequence(seed)))`` created by
``reset(seed=...)`` and continued by later ``reset()`` calls.  The GPU continues that PCG64
stream itself (csrc/spl_rng.h, Pcg64); the host only turns a user seed into the initial PCG64
state — SeedSequence hashing is host-side setup, not per-step work.
"""
import numpy as np

MASK64 = (1 << 64) - 1


def pcg64_state(seed):
    """[state_hi, state_lo, inc_hi, inc_lo] of PCG64(SeedSequence(seed)) (seed None = fresh entropy)."""
    st = np.random.PCG64(np.random.SeedSequence(seed)).state["state"]
    s, inc = int(st["state"]), int(st["inc"])
    return [(s >> 64) & MASK64, s & MASK64, (inc >> 64) & MASK64, inc & MASK64]


def pcg64_states(seeds):
    """uint64[n, 4] PCG64 states for a sequence of seeds (None entries draw fresh entropy)."""
    return np.array([pcg64_state(None if s is None else int(s)) for s in seeds], dtype=np.uint64).reshape(-1, 4)


def vector_seeds(seed, num_envs):
    """gymnasium SyncVectorEnv.reset seed expansion: int -> [seed + i], list kept, None -> None."""
    if seed is None:
        return None
    if isinstance(seed, (int, np.integer)):
        return [int(seed) + i for i in range(num_envs)]
    seeds = list(seed)
    if len(seeds) != num_envs:
        raise ValueError(f"expected {num_envs} seeds, got {len(seeds)}")
    return seeds
