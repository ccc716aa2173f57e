"""Round 5 diagnostic: the device's C5 walks with return_history on
the reference replay fixture (tests/golden/replay_wenner_topography.npz), saved per step so
that the first step leaving the reference's path can be classified on the host
(tools/r05/c5_divergence.py). Usage: c5_hist_dump.py OUT.npz   (WOST_EXP_FLAGS as set)"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)

from dcrmontecarlo_amd import scenarios as S  # noqa: E402
from dcrmontecarlo_amd.geometry import PolyLinesSimple  # noqa: E402
from dcrmontecarlo_amd.solvers import WostSolver_2D  # noqa: E402


def main(out, fixture="replay_wenner_topography.npz", physical=False):
    z = np.load(os.path.join(REPO, "tests", "golden", fixture))
    sc = (S.wenner_topography_physical if physical else S.wenner_topography)(n_walks=1)
    s = WostSolver_2D(PolyLinesSimple(z["dirichlet"]), sc.g, PolyLinesSimple(z["neumann"]), source=sc.f,
                      alpha=sc.alpha)
    W = int(z["n_walks"])
    pts = z["points"]
    u, hist = s.solve(pts, nWalks=W, maxSteps=int(z["max_steps"]), eps=float(z["eps"]), seed=int(z["seed"]),
                      return_history=True)
    walks = [w for i in range(len(pts)) for w in hist[i]]
    P, dd, dn, SP, SV, steps, vals, fin, bnd = [], [], [], [], [], [], [], [], []
    for w in walks:
        steps.append(w["steps"])
        vals.append(w["value"])
        for st in w["path"]:
            P.append(np.asarray(st["point"], np.float32))
            dd.append(st["dirichlet_distance"])
            dn.append(np.nan if st["neumann_distance"] is None else st["neumann_distance"])
        for c in w["contributions"][:-1]:
            SP.append(np.asarray(c["point"], np.float32))
            SV.append(c["contribution"])
        fin.append(np.asarray(w["contributions"][-1]["point"], np.float32))
        bnd.append(w["contributions"][-1]["contribution"])
    np.savez_compressed(out, steps=np.array(steps, np.int64), values=np.array(vals, np.float64),
                        path_points=np.array(P, np.float32).reshape(-1, 2), path_dd=np.array(dd, np.float32),
                        path_dn=np.array(dn, np.float32), src_points=np.array(SP, np.float32).reshape(-1, 2),
                        src_values=np.array(SV, np.float32), final_points=np.array(fin, np.float32).reshape(-1, 2),
                        boundary_values=np.array(bnd, np.float32), sigma_bar=np.float64(s.sigma_bar),
                        flags=np.int64(int(os.environ.get("WOST_EXP_FLAGS", "0"))))
    rs = z["walk_steps"]
    rv = z["walk_values"]
    v = np.array(vals)
    scale = max(float(np.abs(rv).max()), 1e-30)
    same = (np.array(steps) == rs) & (np.abs(v - rv) <= 1e-3 * np.abs(rv) + 1e-5 * scale)
    print(out, "walks", len(steps), "identical to the reference", float(same.mean()), "sigma_bar", s.sigma_bar)


if __name__ == "__main__":
    main(sys.argv[1], *(sys.argv[2:3] or []))
