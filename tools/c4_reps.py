#!/usr/bin/env python3
"""Per-solve walk-kernel time of the C4 bench workload over many back-to-back solves
(is the bench's average held down by clocks under sustained load?)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dcrmontecarlo_amd import scenarios as S  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 30
sc = S.dcr_dipole()
s = sc.solver(device=0)
s.solve(sc.points, nWalks=100_000, maxSteps=sc.max_steps, eps=sc.eps, seed=1)
for k in range(n):
    t0 = time.perf_counter()
    s.solve(sc.points, nWalks=sc.n_walks, maxSteps=sc.max_steps, eps=sc.eps, seed=k)
    w = time.perf_counter() - t0
    t = s.last_timing
    print(f"rep {k:3d} kernel {t['walk_kernel_ms']:.3f} ms  wall {1e3 * w:.3f} ms  "
          f"{t['total_steps'] / (t['walk_kernel_ms'] * 1e-3):.4e} steps/s (kernel)", flush=True)
    if len(sys.argv) > 2:
        time.sleep(float(sys.argv[2]))
