#!/usr/bin/env python3
"""STUDY (host only; round 5): rounds per wave-step of a wave-wide task
pool per Neumann query kind (tools/study/pool_study.cpp) at recorded C5 walk positions
(tests/golden/c5_walk_positions.npz), for waves drawn at random and for waves of the walk
pools' two classes (near the topography / far), against the device's measured issues of
the current per-lane searches with hand-outs (profiles/r04_ab/c5_tree_loop_counters.log:
2.85 silhouette and 4.0 ray record-visit issues and 0.3 + 0.75 leaf rounds per wave-step).
Usage: python tools/study/pool_study.py [lib]"""
import ctypes
import math
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)


def build():
    out = "/tmp/libpool_study.so"
    subprocess.run(["/opt/rocm/bin/hipcc", "-O2", "-std=c++17", "-fPIC", "-shared", "--offload-arch=gfx950",
                    "-ffp-contract=off", "-I" + os.path.join(REPO, "include"), "-x", "hip",
                    os.path.join(REPO, "tools", "study", "pool_study.cpp"), "-x", "c++",
                    os.path.join(REPO, "dcrmontecarlo_amd", "csrc", "wost_tree.cpp"), "-o", out], check=True)
    return out


def main():
    from dcrmontecarlo_amd import scenarios as S

    lib = ctypes.CDLL(sys.argv[1] if len(sys.argv) > 1 else build())
    fp, lp = ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_long)
    lib.pool_wave.argtypes = [fp, ctypes.c_int, ctypes.c_int, fp, fp, fp, ctypes.c_int, ctypes.c_int, lp]
    z = np.load(os.path.join(REPO, "tests", "golden", "c5_walk_positions.npz"))
    P, dd = np.ascontiguousarray(z["points"], np.float32), np.ascontiguousarray(z["dd"], np.float32)
    rng = np.random.default_rng(0)
    th = rng.random(len(P)) * 2 * math.pi
    D = np.ascontiguousarray(np.stack([np.cos(th), np.sin(th)], 1), np.float32)
    V = np.ascontiguousarray(S.topography(10_000), np.float32)
    near = (np.abs(P[:, 0]) <= 600) & (P[:, 1] >= -101) & (P[:, 1] <= 103)   # the pools' box (10% of the extent)
    groups = {"random waves": rng.permutation(len(P)),
              "pooled: near waves": rng.permutation(np.flatnonzero(near)),
              "pooled: far waves": rng.permutation(np.flatnonzero(~near))}
    f = lambda a: a.ctypes.data_as(fp)
    for lifo in (0, 1):
        for name, idx in groups.items():
            idx = idx[: (len(idx) // 64) * 64].reshape(-1, 64)[:300]
            acc = np.zeros(8)
            for w in idx:
                out = np.zeros(8, np.int64)
                p, d, r = (np.ascontiguousarray(a[w]) for a in (P, D, dd))
                assert lib.pool_wave(f(V), V.shape[0], 10, f(p), f(d), f(r), 64, lifo, out.ctypes.data_as(lp)) == 0
                acc += out
            a = acc / len(idx)
            print(f"{'LIFO' if lifo else 'FIFO'} {name:20s} silhouette: {a[0]:.2f} visit rounds ({a[2] / max(a[0], 1e-9):.1f} "
                  f"lanes), {a[1]:.2f} leaf rounds ({a[3] / max(a[1], 1e-9):.1f}); ray: {a[4]:.2f} visit rounds "
                  f"({a[6] / max(a[4], 1e-9):.1f} lanes), {a[5]:.2f} leaf rounds ({a[7] / max(a[5], 1e-9):.1f})")
    print("device, current searches with hand-outs (walk pools on, round 4 counters): silhouette 2.85 visit issues "
          "(19.7 lanes) + 0.3 leaf rounds; ray 4.0 (14.6 lanes) + 0.75 leaf rounds per wave-step")


if __name__ == "__main__":
    main()
