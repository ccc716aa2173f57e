#!/usr/bin/env python3
"""Where a fresh handle's first C4 solve spends its wall time beyond the walk kernel
(bench.py cold.first_solve_ms 64 ms vs the warm 27.8 ms): fresh handles solving the full
call directly, and fresh handles solving a tiny call first (program upload, sampler table,
kernel lookup, small buffers) and the full call next (buffer growth)."""
import json
import sys
import time

sys.path.insert(0, ".")
from dcrmontecarlo_amd import scenarios as S  # noqa: E402


def run(slv, sc, W, seed=7):
    t0 = time.perf_counter()
    slv.solve(sc.points, nWalks=W, maxSteps=sc.max_steps, eps=sc.eps, seed=seed)
    wall = 1e3 * (time.perf_counter() - t0)
    t = slv.last_timing
    return {"wall_ms": round(wall, 2), "total_ms": round(t["total_ms"], 2), "walk_ms": round(t["walk_kernel_ms"], 2),
            "jit_ms": round(t["jit_ms"], 2)}


def main():
    sc = S.ALL["dcr_dipole"]()
    W = 1_000_000
    warm = sc.solver(device=0)
    out = {"warmup": run(warm, sc, W), "warm": [run(warm, sc, W) for _ in range(3)]}
    for i in range(3):
        t0 = time.perf_counter()
        s = sc.solver(device=0)
        c = 1e3 * (time.perf_counter() - t0)
        out[f"fresh{i}"] = {"create_ms": round(c, 2), "first": run(s, sc, W), "second": run(s, sc, W)}
        del s
    for i in range(2):
        s = sc.solver(device=0)
        out[f"tiny_first{i}"] = {"tiny": run(s, sc, 64), "full": run(s, sc, W), "full2": run(s, sc, W)}
        del s
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
