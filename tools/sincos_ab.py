#!/usr/bin/env python3
"""How much of the device/oracle walk disagreement is the hardware sin/cos? Per
scenario: the share of walks identical to the CPU oracle (same Philox streams)
with the kernels' v_sin/v_cos and with the device library's accurate sinf/cosf
(WOST_EXP_FLAGS=128), and the walk-kernel speed of each. Usage (GPU box):
python tools/sincos_ab.py"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dcrmontecarlo_amd import scenarios as S  # noqa: E402
from oracle import oracle as O  # noqa: E402

CASES = [("variable_coefficients", 16, 4096), ("dcr_dipole", 8, 4096), ("notebook_dcr", 8, 4096),
         ("manufactured_polynomial", 16, 4096)]
out = {}
for name, n, W in CASES:
    sc = S.ALL[name]()
    pts = sc.points[:n] if name != "dcr_dipole" else sc.points[20:20 + n]
    row = {}
    for flag in ("0", "128"):
        os.environ["WOST_EXP_FLAGS"] = flag
        s = sc.solver(device=0)
        gv, gs = s.solve_walks(pts, nWalks=W, maxSteps=sc.max_steps, eps=sc.eps, seed=11)
        if flag == "0":
            ov, os_ = O.Problem.from_scenario(sc, sigma_bar=s.sigma_bar or 0.0).solve_walks(
                pts, W, sc.max_steps, sc.eps, 11)
            ov, os_ = ov.reshape(gv.shape), os_.reshape(gs.shape)
        scale = max(float(np.abs(ov).max()), 1e-30)
        same = (gs == os_) & (np.abs(gv - ov) <= 1e-3 * np.abs(ov) + 1e-5 * scale)
        big = S.ALL[name]()
        _, st = s.solve(big.points[:n], nWalks=200_000, maxSteps=sc.max_steps, eps=sc.eps, seed=3, return_stats=True)
        t = s.last_timing
        row[flag] = {"identical_to_oracle": float(same.mean()), "steps_equal": float((gs == os_).mean()),
                     "walk_steps_per_s": t["total_steps"] / (t["walk_kernel_ms"] * 1e-3)}
    out[name] = row
    print(name, json.dumps(row), flush=True)
print("JSON " + json.dumps(out))
