"""the HIP engine under its bounds-check build.  libsplendor_amd_checked.so (same
sources, -DSPL_BOUNDS_CHECK) records table / slot-record / deck / token-table / deal-scratch index
and byte-range violations instead of trusting them; parity workloads of every kernel (steps with
illegal and out-of-range actions, all rollout kernels and player counts, the reference's crafted
edge cases, the MT continuation) must record none.  Runs in ONE child process (the library is
chosen at load time) with the same oracle checks as the main suite."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(os.path.dirname(HERE), "splendor-gym_amd", "splendor_gym", "libsplendor_amd_checked.so")


def test_bounds_check_build_records_no_violation():
    assert os.path.exists(LIB), "build it: python -c 'import __graft_entry__ as g; g.build()'"
    env = dict(os.environ, SPLENDOR_AMD_LIB=LIB)
    r = subprocess.run([sys.executable, os.path.join(HERE, "bounds_check_child.py")], env=env, capture_output=True,
                       text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["steps"] > 500_000
    assert res["flags"] == 0, f"invariant violations recorded: {res['flags']:#x}"
