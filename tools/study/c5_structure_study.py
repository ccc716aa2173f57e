#!/usr/bin/env python3
"""STUDY (host only; round 6): does a structural change to the C5
segment-tree search cut a wave's issue cycles by >= 20%? Per recorded C5 walk position
(tests/golden/c5_walk_positions.npz: 30k positions of device walks, with their Dirichlet
distances) tools/study/c5_structure_study.cpp counts each Neumann query's work under the
current 4-ary tree and under a 16-ary tree; waves of 64 queries are then formed as

  random          the kernels without walk pools
  pools (2)       the kernels' walk pools: near / far waves (wost_walk.h, the default)
  classes (K)     candidate (a): K spatial classes -- 16 or 64 x-bins of the topography
                  over the near box, plus the far class -- so a wave's lanes descend the
                  same subtrees

and priced in child-test rounds (one lane testing one child box = one unit of VALU work;
a 4-ary record visit tests 4):

  4-ary, per lane       4 x max over the wave's queries of record visits (no hand-outs)
  4-ary, ideal sharing  4 x max(ceil(sum visits / 64), longest root-to-leaf chain): the
                        hand-outs (today's kernels) at best -- every lane busy, no query
                        faster than its chain
  16-ary, cooperative   candidate (b): 16 lanes per query test a wide node's 16 children at
                        once: max(ceil(sum child tests / 64), chain) rounds of 1 test

Leaf scans are the same leaves under every layout and are listed, not priced. The device's
round-4 counters (profiles/r04_ab/c5_tree_loop_counters.log: silhouette 2.85 visit issues
with 19.7 lanes, ray 4.0 with 14.6 lanes per wave-step) calibrate the 4-ary rows.
Usage: python tools/study/c5_structure_study.py > profiles/r06_study/c5_structure_study.txt"""
import ctypes
import math
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)


def build():
    out = "/tmp/libc5_structure_study.so"
    subprocess.run(["/opt/rocm/bin/hipcc", "-O2", "-std=c++17", "-fPIC", "-shared", "--offload-arch=gfx950",
                    "-ffp-contract=off", "-I" + os.path.join(REPO, "include"), "-x", "hip",
                    os.path.join(REPO, "tools", "study", "c5_structure_study.cpp"), "-x", "c++",
                    os.path.join(REPO, "dcrmontecarlo_amd", "csrc", "wost_tree.cpp"), "-o", out], check=True)
    return out


def wave_costs(m, idx):
    """Per wave (rows of idx: 64 query indices): child-test rounds of the three searches and
    the leaf scans, for the silhouette (cols 0-3) and the ray query (cols 4-7)."""
    out = {}
    for kind, c in (("silhouette", 0), ("ray", 4)):
        v4, c16, lv, path = (m[idx, c + k].astype(np.float64) for k in range(4))
        per_lane = 4.0 * v4.max(1)
        ideal4 = 4.0 * np.maximum(np.ceil(v4.sum(1) / 64.0), path.max(1))
        chain16 = np.ceil(path.max(1) / 2.0)            # a wide node spans two 4-ary levels
        ideal16 = np.maximum(np.ceil(c16.sum(1) / 64.0), chain16)
        out[kind] = {"visits": v4.sum(1).mean(), "lanes_per_visit_round": (v4.sum(1) / np.maximum(v4.max(1), 1)).mean(),
                     "per_lane": per_lane.mean(), "ideal4": ideal4.mean(), "ideal16": ideal16.mean(),
                     "child_tests4": 4.0 * v4.sum(1).mean(), "child_tests16": c16.sum(1).mean(),
                     "leaves": lv.sum(1).mean()}
    return out


def main():
    from dcrmontecarlo_amd import scenarios as S

    lib = ctypes.CDLL(sys.argv[1] if len(sys.argv) > 1 else build())
    fp, lp = ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_long)
    lib.structure_queries.argtypes = [fp, ctypes.c_int, ctypes.c_int, fp, fp, fp, ctypes.c_int, lp]
    z = np.load(os.path.join(REPO, "tests", "golden", "c5_walk_positions.npz"))
    P, dd = np.ascontiguousarray(z["points"], np.float32), np.ascontiguousarray(z["dd"], np.float32)
    rng = np.random.default_rng(0)
    th = rng.random(len(P)) * 2 * math.pi
    D = np.ascontiguousarray(np.stack([np.cos(th), np.sin(th)], 1), np.float32)
    V = np.ascontiguousarray(S.topography(10_000), np.float32)
    f = lambda a: a.ctypes.data_as(fp)
    m = np.zeros((len(P), 8), np.int64)
    assert lib.structure_queries(f(V), V.shape[0], 10, f(P), f(D), f(dd), len(P), m.ctypes.data_as(lp)) == 0
    print(f"{len(P)} recorded C5 walk positions, 10,000-segment topography, leaves of 10 segments")
    for kind, c in (("silhouette", 0), ("ray", 4)):
        v = m[:, c]
        print(f"  {kind:10s}: record visits per query mean {v.mean():.2f}, p50 {np.median(v):.0f}, p90 "
              f"{np.percentile(v, 90):.0f}, max {v.max()}; queries with <= 2 visits {np.mean(v <= 2):.3f}; "
              f"child tests per query 4-ary {4 * v.mean():.2f}, 16-ary {m[:, c + 1].mean():.2f}; "
              f"leaves {m[:, c + 2].mean():.2f}")
    near = (np.abs(P[:, 0]) <= 600) & (P[:, 1] >= -101) & (P[:, 1] <= 103)   # the pools' box (10% of the extent)
    x0, x1 = float(V[:, 0].min()), float(V[:, 0].max())

    def classes(k):
        b = np.clip(((P[:, 0] - x0) / (x1 - x0) * k).astype(np.int64), 0, k - 1)
        return np.where(near, b, k)                                   # class k: far

    def waves(labels):
        rows = []
        for c in np.unique(labels):
            ii = rng.permutation(np.flatnonzero(labels == c))
            rows += [ii[i:i + 64] for i in range(0, len(ii) - 63, 64)]
        return np.array(rows)

    groups = {"random": waves(np.zeros(len(P), np.int64)), "pools (2)": waves(near.astype(np.int64)),
              "classes (16)": waves(classes(16)), "classes (64)": waves(classes(64))}
    print("\nper wave-step (waves of 64 queries; child-test rounds, one child box per lane per round)")
    base = {}
    for name, idx in groups.items():
        w = wave_costs(m, idx)
        for kind in ("silhouette", "ray"):
            r = w[kind]
            print(f"  {name:13s} {kind:10s}: visits {r['visits']:6.1f} ({r['lanes_per_visit_round']:5.1f} lanes per "
                  f"per-lane round) | 4-ary per lane {r['per_lane']:6.1f}  4-ary ideal sharing {r['ideal4']:5.1f}  "
                  f"16-ary cooperative {r['ideal16']:5.1f} | child tests 4-ary {r['child_tests4']:6.1f} 16-ary "
                  f"{r['child_tests16']:6.1f} | leaves {r['leaves']:5.1f}")
        base[name] = w
    print("\nverdict (against the kernels' design, pools (2) with sharing -- the 4-ary ideal row):")
    p = base["pools (2)"]
    tot4 = p["silhouette"]["ideal4"] + p["ray"]["ideal4"]
    for name in ("classes (16)", "classes (64)"):
        t = base[name]["silhouette"]["ideal4"] + base[name]["ray"]["ideal4"]
        print(f"  (a) {name}: {t:.1f} vs {tot4:.1f} child-test rounds per wave-step ({100 * (1 - t / tot4):+.1f}% "
              f"fewer); per lane without sharing {base[name]['silhouette']['per_lane'] + base[name]['ray']['per_lane']:.1f} "
              f"vs {p['silhouette']['per_lane'] + p['ray']['per_lane']:.1f}")
    t16 = p["silhouette"]["ideal16"] + p["ray"]["ideal16"]
    print(f"  (b) 16-ary cooperative nodes: {t16:.1f} vs {tot4:.1f} ({100 * (1 - t16 / tot4):+.1f}% fewer); total "
          f"child tests {p['silhouette']['child_tests16'] + p['ray']['child_tests16']:.0f} vs "
          f"{p['silhouette']['child_tests4'] + p['ray']['child_tests4']:.0f} (4-ary)")
    print("  build threshold: >= 20% fewer issue cycles (VERDICT r05)")
    print("device, round-4 counters: silhouette 2.85 visit issues (19.7 lanes), ray 4.0 (14.6 lanes) per wave-step, "
          "i.e. 56 and 58 record visits: 4 x (2.85 + 4.0) = 27.4 child-test rounds")


if __name__ == "__main__":
    main()
