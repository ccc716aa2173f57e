#!/usr/bin/env python3
"""A fresh process's first solve, phase by phase (the reference's usage: one solve per
script): import, handle creation, the first solve (its kernel in no cache: jit_race), the
second; and the compile helper's own start (wost_jitc --identity). Usage:
cold_first_solve.py <scenario> <points> <walks> [jit_race]"""
import json
import os
import subprocess
import sys
import tempfile
import time

t_start = time.perf_counter()
d = tempfile.mkdtemp(prefix="wost_cold1_")
os.environ["WOST_JIT_CACHE"] = d
os.environ["AMD_COMGR_CACHE_DIR"] = os.path.join(d, "comgr")
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from dcrmontecarlo_amd import _lib  # noqa: E402
from dcrmontecarlo_amd import scenarios as S  # noqa: E402


def main():
    name, n, W = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    race = int(sys.argv[4]) if len(sys.argv) > 4 else 1
    out = {"scenario": name, "points": n, "walks": W, "jit_race": race,
           "import_ms": 1e3 * (time.perf_counter() - t_start)}
    t0 = time.perf_counter()
    sc = S.ALL[name]()
    s = sc.solver(device=0)
    s.set_option("jit_race", race)
    out["create_ms"] = 1e3 * (time.perf_counter() - t0)
    for k in range(3):
        t0 = time.perf_counter()
        s.solve(sc.points[:n], nWalks=W, maxSteps=sc.max_steps, eps=sc.eps, seed=7)
        t = s.last_timing
        out[f"solve{k}"] = {"wall_ms": 1e3 * (time.perf_counter() - t0), "libwost_ms": t["total_ms"],
                            "walk_kernel_ms": t["walk_kernel_ms"], "jit_ms": t["jit_ms"], "jit": t["jit"],
                            "precompiled_walks": t["precompiled_walks"], "launches": t["n_launches"]}
    helper = os.path.join(os.path.dirname(_lib.LIB_PATH), "wost_jitc")
    t0 = time.perf_counter()
    subprocess.run([helper, "--identity"], check=True, capture_output=True)
    out["helper_identity_ms"] = 1e3 * (time.perf_counter() - t0)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
