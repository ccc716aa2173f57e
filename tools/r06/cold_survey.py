#!/usr/bin/env python3
"""The C5 survey's cold start: a fresh process's first Wenner survey
(256 electrodes, 3 handle pairs as bench.py runs it) with an empty kernel cache and an
empty comgr cache, its kernels compiled in helper processes (option jit_process = 1, the
default) or in this process (0), then a warm survey. Usage: cold_survey.py <0|1> [walks]"""
import json
import os
import sys
import tempfile
import time

d = tempfile.mkdtemp(prefix="wost_cold_")
os.environ["WOST_JIT_CACHE"] = d
os.environ["AMD_COMGR_CACHE_DIR"] = os.path.join(d, "comgr")
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from dcrmontecarlo_amd import scenarios as S  # noqa: E402
from dcrmontecarlo_amd import survey  # noqa: E402

ALPHA_BG = 0.01


def main():
    proc = int(sys.argv[1])
    W = int(sys.argv[2]) if len(sys.argv) > 2 else 100_000
    t0 = time.perf_counter()
    sc = S.wenner_topography(n_electrodes=256, n_walks=W)
    pairs = []
    for _ in range(3):
        m = sc.solver(device=0)
        pairs += [m, survey.homogeneous_solver(sc, ALPHA_BG, m, device=0)]
    for s in pairs:
        s.set_option("jit_process", proc)
    setup = time.perf_counter() - t0
    out = {"jit_process": proc, "walks": W, "setup_ms": 1e3 * setup}
    for k in range(3):
        ts = time.perf_counter()
        r = survey.run_wenner_survey(sc, ALPHA_BG, W, seed=1000 + k, solvers=tuple(pairs))
        out[f"survey{k}_ms"] = 1e3 * (time.perf_counter() - ts)
        out[f"survey{k}_steps"] = int(r.walk_steps)
    out["kernels_cached"] = len([f for f in os.listdir(d) if f.endswith(".hsaco")])
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
