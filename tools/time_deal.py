"""Time the deal kernels (k_refill, k_reset) against the number of tables dealt.

    python tools/time_deal.py        # on the GPU box
A fresh arena has every table pending (unseeded: engine seed 0), so spl_refill deals all n
tables: the curve over n separates per-wave latency (flat region) from throughput (linear).
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "splendor-gym_amd")]

import torch  # noqa: E402

from splendor_gym import _native  # noqa: E402
from splendor_gym.device import Engine  # noqa: E402


def timed(fn, reps=5):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    out = []
    for _ in range(reps):
        fn()
        torch.cuda.synchronize()
    for _ in range(reps):
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        out.append(s.elapsed_time(e) * 1000)
    return min(out), sorted(out)[len(out) // 2]


def main():
    for n in (64, 1024, 4096, 16384, 65536, 262144):
        e = Engine(n, 2, device="cuda:0", refill_period=0)
        import ctypes
        lib, ar = e.lib, ctypes.byref(e.desc)

        def refill_all():
            _native.check(lib, lib.spl_arena_init(e.ctx, ar, e.stream()))
            _native.check(lib, lib.spl_refill(e.ctx, ar, e.stream()))

        def init_only():
            _native.check(lib, lib.spl_arena_init(e.ctx, ar, e.stream()))
        base = timed(init_only)
        r = timed(refill_all)
        s = timed(lambda: e.reset(seeds=range(n)))
        print(f"n={n:7d}  refill(all pending) {r[1] - base[1]:8.1f} us   reset(seeded, 2 deals) {s[1]:8.1f} us",
              flush=True)
        e.close()


if __name__ == "__main__":
    main()
