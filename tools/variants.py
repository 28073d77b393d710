"""Experiment builds of the engine library (not the product): each variant is the same sources
compiled with extra -D flags into splendor-gym_amd/ablate/lib_<name>.so (git-ignored), selected at
run time with SPLENDOR_AMD_LIB.  Ablated variants compute wrong outputs by design; only their
timings mean anything.

    python tools/variants.py build name=-DFLAG[,-DFLAG2] ...
    python tools/variants.py bench name ... [-- bench.py args]     (on the GPU box)
"""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "splendor-gym_amd", "csrc")
OUTD = os.path.join(REPO, "splendor-gym_amd", "ablate")
SRCS = [os.path.join(CSRC, f) for f in ("spl_engine.hip", "spl_policy.hip", "spl_policy32.hip", "spl_dual.hip")]


def sources_at(rev):
    """The engine sources as of git revision `rev` (exported to a temporary tree)."""
    import tempfile
    d = tempfile.mkdtemp(prefix="spl_rev_")
    arc = subprocess.run(["git", "-C", REPO, "archive", rev, "splendor-gym_amd/csrc", "include"], check=True,
                         capture_output=True).stdout
    subprocess.run(["tar", "-x", "-C", d], input=arc, check=True)
    return [os.path.join(d, "splendor-gym_amd", "csrc", os.path.basename(f)) for f in SRCS]


def build(specs):
    """name=-DFLAG,... builds the working tree; name@REV=-DFLAG,... builds git revision REV."""
    os.makedirs(OUTD, exist_ok=True)
    procs = []
    for spec in specs:
        name, _, flags = spec.partition("=")
        name, _, rev = name.partition("@")
        srcs = sources_at(rev) if rev else SRCS
        out = os.path.join(OUTD, f"lib_{name}.so")
        cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-w",
               *[f for f in flags.split(",") if f], "-shared", "-o", out, *srcs]
        procs.append((name, subprocess.Popen(cmd)))
    for name, p in procs:
        if p.wait() != 0:
            raise SystemExit(f"build of {name} failed")
        print("built", name)


def bench(names, extra):
    for name in names:
        env = dict(os.environ, SPLENDOR_AMD_LIB=os.path.join(OUTD, f"lib_{name}.so"))
        r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--no-cpu-baseline", *extra], env=env,
                           capture_output=True, text=True, timeout=600)
        if r.returncode != 0:
            print(name, "FAILED", r.stderr[-2000:])
            raise SystemExit(1)
        import json
        d = json.loads(r.stdout.strip().splitlines()[-1])
        line = {"variant": name, "value": d["value"], "kernel_us": d["roofline"]["kernel_avg_us"],
                "frac": d["roofline"]["frac"]}
        for k in ("in_place_l3", "other_mode", "rollout_store"):
            if k in d:
                line[k + "_us"] = d[k]["roofline"]["kernel_avg_us"]
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build(sys.argv[2:])
    else:
        args = sys.argv[2:]
        extra = args[args.index("--") + 1:] if "--" in args else []
        names = args[:args.index("--")] if "--" in args else args
        bench(names, extra)
