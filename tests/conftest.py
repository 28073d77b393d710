"""pytest configuration: markers and import paths.

`-m "not gpu"` runs here (no GPU): oracle vs golden fixtures, host logic, ABI exports, gloo.
`-m gpu` runs on an MI355X box: HIP engine parity against the oracle.
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "splendor-gym_amd"), os.path.join(REPO, "tests", "golden")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running")
