"""Round 5 diagnostic: where each C5 walk of a device history dump (tools/r05/c5_hist_dump.py)
first leaves the reference's replayed path (tests/golden/replay_wenner_topography.npz).
For every walk whose step count or value differs, the first step j whose point, Dirichlet
or silhouette distance differs from the reference's, classified by the transition j-1 -> j:
  distance   the query distances at j-1 already differ (dd / dn)
  direction  the source sample point at j-1 differs (direction or sampled radius)
  collision  same sample point, but one walk moved to it and the other to the ray's point
  ray        same sample point and both moved to the ray's point, which differs (hit test)
  sample     both collided, at different points (cannot happen if the samples agree)
Usage: c5_divergence.py HIST.npz [fixture]"""
import os
import sys
from collections import Counter

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def ulps(a, b):
    a, b = np.asarray(a, np.float32), np.asarray(b, np.float32)
    m = np.maximum(np.maximum(np.abs(a), np.abs(b)), np.float32(1e-30))
    return np.where((a == b) | (np.isnan(a) & np.isnan(b)), 0.0, np.abs(a.astype(np.float64) - b) / np.spacing(m))


def analyse(hist, z, tol_ulp=0.0, verbose=False):
    rs, rv = z["walk_steps"], z["walk_values"]
    gs, gv = hist["steps"], hist["values"]
    scale = max(float(np.abs(rv).max()), 1e-30)
    same = (gs == rs) & (np.abs(gv - rv) <= 1e-3 * np.abs(rv) + 1e-5 * scale)
    ro = np.concatenate([[0], np.cumsum(rs)])
    go = np.concatenate([[0], np.cumsum(gs)])
    kinds = Counter()
    rows = []
    for w in range(len(rs)):
        n = min(rs[w], gs[w])
        RP, GP = z["path_points"][ro[w]:ro[w] + n], hist["path_points"][go[w]:go[w] + n]
        Rd, Gd = z["path_dd"][ro[w]:ro[w] + n], hist["path_dd"][go[w]:go[w] + n]
        Rn, Gn = z["path_dn"][ro[w]:ro[w] + n], hist["path_dn"][go[w]:go[w] + n]
        RS, GS = z["src_points"][ro[w]:ro[w] + n], hist["src_points"][go[w]:go[w] + n]
        bad = (ulps(RP, GP).max(1) > tol_ulp) | (ulps(Rd, Gd) > tol_ulp) | (ulps(Rn, Gn) > tol_ulp)
        if not bad.any():
            if not same[w]:
                kinds["end (steps or boundary term)"] += 1
            continue
        j = int(np.argmax(bad))
        if j == 0:
            kind = "start"
        else:
            i = j - 1
            if ulps(Rd[i], Gd[i]) > tol_ulp or ulps(Rn[i], Gn[i]) > tol_ulp:
                kind = "distance"
            elif ulps(RS[i], GS[i]).max() > tol_ulp:
                kind = "direction"
            else:
                r_col = bool(np.all(RP[j] == RS[i]))
                g_col = bool(np.all(GP[j] == GS[i]))
                kind = "collision" if r_col != g_col else ("sample" if r_col else "ray")
        kinds[kind] += 1
        rows.append((w, j, kind, bool(same[w])))
        if verbose:
            print(w, "first divergent step", j, kind, "walk identical" if same[w] else "walk differs",
                  "ref", RP[j].tolist(), "dev", GP[j].tolist())
    return float(same.mean()), kinds, rows


if __name__ == "__main__":
    fx = sys.argv[2] if len(sys.argv) > 2 else os.path.join(REPO, "tests", "golden", "replay_wenner_topography.npz")
    z = np.load(fx)
    h = np.load(sys.argv[1])
    agree, kinds, rows = analyse(h, z, verbose="-v" in sys.argv)
    diff = [r for r in rows if not r[3]]
    print(f"{sys.argv[1]}: walks identical to the reference {agree:.4f}; paths leaving the reference's "
          f"(any step, 0 ulp): {len(rows)}; of the differing walks, first divergence: "
          f"{dict(Counter(r[2] for r in diff))}; all: {dict(kinds)}")
