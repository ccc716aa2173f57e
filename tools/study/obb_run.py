#!/usr/bin/env python3
"""STUDY: OBB segment-tree visit counts vs the AABB tree at the C5 walk positions
(/tmp/c5_counts.npz from c5_wave_study.py); exactness against the full scans."""
import ctypes
import sys

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from dcrmontecarlo_amd import scenarios as S  # noqa: E402

lib = ctypes.CDLL(sys.argv[1] if len(sys.argv) > 1 else "/tmp/libobb_study.so")
fp = ctypes.POINTER(ctypes.c_float)
lp = ctypes.POINTER(ctypes.c_long)
lib.obb_counts.argtypes = [fp, ctypes.c_int, ctypes.c_int, ctypes.c_float, fp, fp, fp, ctypes.c_float, ctypes.c_float,
                           ctypes.c_long, lp, lp, ctypes.c_int]
z = np.load("/tmp/c5_counts.npz")
P, D, dd, base = [np.ascontiguousarray(z[k]) for k in ("points", "dirs", "dd", "counts")]
V = np.ascontiguousarray(S.topography(10_000), np.float32)
rmin = np.float32(0.45)
stop2 = np.float32(0.2025)
while np.sqrt(np.float32(np.nextafter(stop2, np.float32(1)))) <= rmin:
    stop2 = np.nextafter(stop2, np.float32(1))
while np.sqrt(stop2) > rmin:
    stop2 = np.nextafter(stop2, np.float32(0))
leaf = int(sys.argv[2]) if len(sys.argv) > 2 else 8
margin = float(sys.argv[3]) if len(sys.argv) > 3 else 1e-5
arity = int(sys.argv[4]) if len(sys.argv) > 4 else 2
n = len(P)
out = np.zeros((n, 4), np.int64)
mism = np.zeros(2, np.int64)
lib.obb_counts(V.ctypes.data_as(fp), V.shape[0], leaf, margin, P.ctypes.data_as(fp), D.ctypes.data_as(fp),
               dd.ctypes.data_as(fp), rmin, stop2, n, out.ctypes.data_as(lp), mism.ctypes.data_as(lp), arity)
print("leaf", leaf, "margin", margin, "arity", arity, "mismatches (r, ray):", mism.tolist())
rng = np.random.default_rng(0)
perm = rng.permutation(n)[: (n // 64) * 64].reshape(-1, 64)
for k, nm in enumerate(["sil_rec", "sil_leaf", "ray_rec", "ray_leaf"]):
    for lab, c in (("aabb", base[:, k]), ("obb ", out[:, k])):
        w = c[perm]
        print(f"{nm:9s} {lab} mean {c.mean():6.2f} p99 {np.percentile(c, 99):5.0f} max {c.max():5d}   wave max-mean "
              f"{w.max(1).mean():6.2f}")
