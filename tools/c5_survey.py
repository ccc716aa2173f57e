#!/usr/bin/env python3
"""C5 (BASELINE configs[4]): the 256-electrode Wenner line over the 10,000-segment
topography, model and homogeneous background, multi-source batched
(survey.run_wenner_survey). Prints walk-steps/s (walk-kernel time and wall time),
the launches, and the apparent-resistivity summary as one JSON line.
Usage: python tools/c5_survey.py [--walks 4096] [--a 1]"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--walks", type=int, default=4096)
    ap.add_argument("--a", type=int, default=1)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--serial", action="store_true", help="model and background one after the other")
    a = ap.parse_args()
    from dcrmontecarlo_amd import scenarios as S
    from dcrmontecarlo_amd import survey

    sc = S.wenner_topography(n_electrodes=256, n_walks=a.walks)
    sm = sc.solver(device=0)
    sh = survey.homogeneous_solver(sc, 1e-2, sm, device=0)
    survey.run_wenner_survey(sc, 1e-2, n_walks=64, a=a.a, seed=a.seed + 1, solvers=(sm, sh))   # warm-up / JIT
    t0 = time.perf_counter()
    res = survey.run_wenner_survey(sc, 1e-2, n_walks=a.walks, a=a.a, seed=a.seed, solvers=(sm, sh),
                                   concurrent=not a.serial)
    wall = time.perf_counter() - t0
    ok = res.rho.resolved & np.isfinite(res.rho.rho_a)
    out = {"workload": "C5 Wenner-alpha line, 256 electrodes, 10k-segment topography (notebook fields), "
                       "model + homogeneous background", "a": a.a, "walks_per_electrode": a.walks,
           "quadripoles": int(len(res.quadripoles)), "launches_per_field": res.launches,
           "walk_steps": res.walk_steps, "walk_kernel_ms": res.kernel_ms, "wall_s": wall,
           "walk_steps_per_s_kernel": res.walk_steps / (res.kernel_ms * 1e-3),
           "walk_steps_per_s_wall": res.walk_steps / wall, "concurrent_fields": not a.serial,
           "rho_a": {"resolved": int(ok.sum()), "median": float(np.median(res.rho.rho_a[ok])) if ok.any() else None,
                     "mc_1sigma_rms": float(np.sqrt(np.mean(res.rho.se[ok] ** 2))) if ok.any() else None}}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
