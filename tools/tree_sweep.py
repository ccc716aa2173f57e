#!/usr/bin/env python3
"""Neumann segment tree vs full scan: walk-steps/s of the C5 topography problem
over polyline sizes and leaf sizes (picks WOST_TREE_MIN_SEGMENTS_DEFAULT and
WOST_TREE_LEAF_DEFAULT). Usage: python tools/tree_sweep.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dcrmontecarlo_amd import scenarios as S  # noqa: E402


def rate(sc, W, min_segments, leaf=0):
    s = sc.solver(device=0)
    s.set_segment_tree(min_segments, leaf)
    s.solve(sc.points, nWalks=max(1, W // 8), maxSteps=sc.max_steps, eps=sc.eps, seed=1)
    best = 0.0
    for r in range(2):
        s.solve(sc.points, nWalks=W, maxSteps=sc.max_steps, eps=sc.eps, seed=10 + r)
        t = s.last_timing
        best = max(best, t["total_steps"] / (t["walk_kernel_ms"] * 1e-3))
    return best


def main():
    out = {"size": {}, "leaf": {}}
    for nseg in (4, 8, 16, 32, 64, 128, 256, 1024, 10_000):
        sc = S.wenner_topography(n_electrodes=256, n_walks=1, n_segments=nseg)
        W = 2000
        scan = rate(sc, W if nseg <= 256 else max(16, W * 256 // nseg), -1) if nseg <= 1024 else None
        tree = rate(sc, W, 0)
        out["size"][nseg] = {"scan": scan, "tree": tree}
        print(f"nseg {nseg:6d}: scan {scan or 0:.3e}  tree {tree:.3e} steps/s", flush=True)
    sc = S.wenner_topography(n_electrodes=256, n_walks=1, n_segments=10_000)
    for leaf in (2, 4, 8, 16, 32, 64):
        out["leaf"][leaf] = rate(sc, 2000, 0, leaf)
        print(f"leaf {leaf:3d}: tree {out['leaf'][leaf]:.3e} steps/s", flush=True)
    print("JSON " + json.dumps(out))


if __name__ == "__main__":
    main()
