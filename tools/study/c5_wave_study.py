#!/usr/bin/env python3
"""STUDY (host only): per-query segment-tree visit counts at the positions C5 walks
visit (gpurun_out/c5_paths.npz from tools/c5_paths.py), and what a wave of 64 lanes
pays for them (max over lanes) versus the mean -- the divergence the tree kernel
suffers. Usage: python tools/study/c5_wave_study.py [lib]"""
import ctypes
import math
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)


def main():
    from dcrmontecarlo_amd import scenarios as S

    lib = ctypes.CDLL(sys.argv[1] if len(sys.argv) > 1 else "/tmp/libtree_study.so")
    fp = ctypes.POINTER(ctypes.c_float)
    lp = ctypes.POINTER(ctypes.c_long)
    lib.tree_counts.argtypes = [fp, ctypes.c_int, ctypes.c_int, fp, fp, fp, ctypes.c_float, ctypes.c_float,
                                ctypes.c_long, lp, fp]
    z = np.load(os.path.join(REPO, "gpurun_out", "c5_paths.npz"))
    P = np.ascontiguousarray(z["points"], np.float32)
    dd = np.ascontiguousarray(z["dd"], np.float32)
    n = len(P)
    rng = np.random.default_rng(0)
    th = rng.random(n) * 2 * math.pi
    D = np.ascontiguousarray(np.stack([np.cos(th), np.sin(th)], 1), np.float32)
    V = np.ascontiguousarray(S.topography(10_000), np.float32)
    rmin = np.float32(0.45)
    stop2 = np.nextafter(rmin * rmin, np.float32(0))
    while math.sqrt(float(np.nextafter(stop2, np.float32(1)))) <= rmin:
        stop2 = np.nextafter(stop2, np.float32(1))
    out = np.zeros((n, 4), np.int64)
    res = np.zeros((n, 2), np.float32)
    rc = lib.tree_counts(V.ctypes.data_as(fp), V.shape[0], int(os.environ.get("LEAF", "8")), P.ctypes.data_as(fp),
                         D.ctypes.data_as(fp), dd.ctypes.data_as(fp), ctypes.c_float(rmin), ctypes.c_float(stop2),
                         n, out.ctypes.data_as(lp), res.ctypes.data_as(fp))
    assert rc == 0
    names = ["sil_rec", "sil_leaf", "ray_rec", "ray_leaf"]
    for k, nm in enumerate(names):
        c = out[:, k]
        print(f"{nm:9s} mean {c.mean():7.2f}  p50 {np.percentile(c, 50):5.0f} p90 {np.percentile(c, 90):5.0f} "
              f"p99 {np.percentile(c, 99):6.0f} max {c.max():6d}")
    # waves: 64 random queries (a wave's lanes hold unrelated walks)
    perm = rng.permutation(n)[: (n // 64) * 64].reshape(-1, 64)
    for k, nm in enumerate(names):
        c = out[perm, k]
        print(f"wave {nm:9s} mean-of-lanes {c.mean():7.2f}  mean max-over-lanes {c.max(1).mean():7.2f}  "
              f"ratio {c.max(1).mean() / max(c.mean(), 1e-9):5.2f}")
    far = np.abs(P[:, 1]) > 1000
    print("far walkers (|y| > 1000):", far.mean(), "their mean ray recs", out[far, 2].mean(), "near", out[~far, 2].mean())
    print("hit fraction", res[:, 1].mean())
    np.savez_compressed("/tmp/c5_counts.npz", counts=out, res=res, points=P, dd=dd, dirs=D)


if __name__ == "__main__":
    main()
