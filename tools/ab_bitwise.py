#!/usr/bin/env python3
"""Bitwise A/B of two libwost builds: every scenario's per-walk values and step counts
must be identical (an optimisation that claims to be exact is checked walk for walk).
Usage (GPU box): python tools/ab_bitwise.py ab/libwost_old.so dcrmontecarlo_amd/libwost.so
Each library runs in its own process (WOST_LIB); prints one line per scenario.
A library argument may carry environment settings for its process:
lib.so:WOST_JIT_SLP=1 (several joined by commas)."""
import json
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SIZES = {"laplace_square": (16, 4096), "manufactured_polynomial": (16, 4096), "poisson_square": (16, 4096),
         "variable_coefficients": (16, 4096), "dcr_dipole": (48, 16384), "notebook_dcr": (21, 4096),
         "wenner_topography": (64, 2048), "wenner_topography_physical": (64, 2048)}


def run_one(out):
    sys.path.insert(0, REPO)
    from dcrmontecarlo_amd import scenarios as S

    res = {}
    for name, (n, W) in SIZES.items():
        sc = S.ALL[name]()
        s = sc.solver(device=0)
        pts = sc.points[:n] if not name.startswith("wenner_topography") else sc.points[::4][:n]
        v, st = s.solve_walks(pts, nWalks=W, maxSteps=sc.max_steps, eps=sc.eps, seed=777)
        res[name + "_v"] = v
        res[name + "_s"] = st
    np.savez(out, **res)


def main():
    if sys.argv[1] == "--one":
        run_one(sys.argv[2])
        return
    outs = []
    for i, arg in enumerate(sys.argv[1:3]):
        lib, _, extra = arg.partition(":")
        out = os.path.join(REPO, "gpurun_out", f"ab_bitwise_{i}.npz")
        env = dict(os.environ, WOST_LIB=os.path.abspath(lib))
        env.update(kv.split("=", 1) for kv in extra.split(",") if kv)
        subprocess.run([sys.executable, os.path.abspath(__file__), "--one", out], check=True, env=env)
        outs.append(np.load(out))
    ok_all = True
    for name in SIZES:
        v0, v1 = outs[0][name + "_v"], outs[1][name + "_v"]
        s0, s1 = outs[0][name + "_s"], outs[1][name + "_s"]
        same_v = np.array_equal(v0.view(np.uint32), v1.view(np.uint32))
        same_s = np.array_equal(s0, s1)
        ok_all &= same_v and same_s
        print(json.dumps({"scenario": name, "walks": int(v0.size), "values_bitwise_equal": bool(same_v),
                          "steps_equal": bool(same_s), "differing_walks": int(np.sum(v0.view(np.uint32) != v1.view(np.uint32)))}))
    print("ALL_BITWISE_EQUAL" if ok_all else "DIFFERENT")


if __name__ == "__main__":
    main()
