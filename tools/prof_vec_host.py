"""Host-side cost of the pieces of SplendorVectorEnv.step (no device syncs inside the timed calls):
python tools/prof_vec_host.py"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "splendor-gym_amd")]
import torch  # noqa: E402
from splendor_gym import SplendorVectorEnv, _native  # noqa: E402

vec = SplendorVectorEnv(65536, device="cuda:0", check_actions="deferred")
vec.reset(seed=0)
e = vec.engine
acts = vec.sample_actions(seed=1, ply=0).clone()
N = 200
def t(name, fn):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(N):
        fn()
    dt = (time.perf_counter() - t0) / N
    torch.cuda.synchronize()
    print(f"{name:40s} {dt * 1e6:8.2f} us host")
t("sample_actions", lambda: vec.sample_actions(seed=1, ply=3))
t("engine.step", lambda: e.step(acts, autoreset=True, final_obs=True))
fl = e.flags
t("bits = (flags[:,None] & b) != 0", lambda: (fl.unsqueeze(1) & vec._bits) != 0)
b = (fl.unsqueeze(1) & vec._bits) != 0
t("bits[:,3].any()", lambda: b[:, 3].any())
t("term.view(bool)", lambda: e.terminated.view(torch.bool))
t("obs[:,294]", lambda: e.obs[:, 294])
t("torch.cuda.current_stream", lambda: torch.cuda.current_stream(e.device))
t("engine.stream()", lambda: e.stream())
t("torch.cuda.current_device", lambda: torch.cuda.current_device())
t("vec.step (deferred)", lambda: vec.step(acts))
vec2 = SplendorVectorEnv(65536, device="cuda:0", check_actions="sync")
vec2.reset(seed=0)
t("vec.step (sync)", lambda: vec2.step(acts))
