#!/usr/bin/env python3
"""Precompiled (interpreting) walk kernel against the field-specialised one, per BASELINE
config, warm: is running a fresh handle's first solve on the precompiled kernel (no
hiprtc compile) worth it? Prints kernel ms and walk-steps/s of both, and a fresh handle's
first-solve wall time with an empty kernel cache."""
import json
import os
import sys
import tempfile
import time

d = tempfile.mkdtemp(prefix="wost_pre_")
os.environ["WOST_JIT_CACHE"] = d
os.environ["AMD_COMGR_CACHE_DIR"] = os.path.join(d, "comgr")
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from dcrmontecarlo_amd import scenarios as S  # noqa: E402

CASES = [("poisson_square", 64, 10_000), ("variable_coefficients", 256, 100_000), ("dcr_dipole", 48, 1_000_000),
         ("laplace_square", 64, 1000), ("wenner_topography", 256, 2000)]


def run(s, sc, n, W, seed=7):
    t0 = time.perf_counter()
    _, st = s.solve(sc.points[:n], nWalks=W, maxSteps=sc.max_steps, eps=sc.eps, seed=seed, return_stats=True)
    return 1e3 * (time.perf_counter() - t0), st.kernel_ms, st.total_steps, s.last_timing["jit_ms"]


def main():
    out = {}
    for name, n, W in CASES:
        sc = S.ALL[name]()
        r = {}
        first = sc.solver(device=0)
        r["jit_first_wall_ms"], _, _, r["jit_first_compile_ms"] = run(first, sc, n, W)
        for jit in (True, False):
            s = sc.solver(device=0)
            s.set_jit(jit)
            w0 = run(s, sc, n, W)
            reps = [run(s, sc, n, W) for _ in range(3)]
            best = min(reps, key=lambda x: x[1])
            tag = "jit" if jit else "pre"
            r[f"{tag}_first_wall_ms"] = w0[0]
            r[f"{tag}_kernel_ms"] = best[1]
            r[f"{tag}_steps_per_s"] = best[2] / (best[1] * 1e-3)
        r["pre_over_jit_kernel"] = r["pre_kernel_ms"] / r["jit_kernel_ms"]
        out[name] = r
        print(name, json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
