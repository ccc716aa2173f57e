"""Round 5: what the direction's trig buys in parity (wost_set_trig), per scenario: the share
of walks identical to the oracle's (correctly rounded cos/sin, the host's atan2f) and to the
reference's replayed walks (tests/golden/replay_*.npz), with exact and with fast (hardware)
trig. Usage: trig_parity.py [scenario ...]"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

from dcrmontecarlo_amd import scenarios as S  # noqa: E402
from oracle import oracle as O  # noqa: E402


def same(v, s, rv, rs):
    scale = max(float(np.abs(rv).max()), 1e-30)
    return float(((np.asarray(s) == rs) & (np.abs(np.asarray(v, np.float64) - rv) <= 1e-3 * np.abs(rv) + 1e-5 * scale)).mean())


def main(names):
    from test_gpu_parity import _solver_for
    from test_oracle_golden import SENS_SIZES, sensitivity_points

    for name in names:
        z = np.load(os.path.join(REPO, "tests", "golden", f"replay_{name}.npz"))
        for trig in ("exact", "fast"):
            sc, s = _solver_for(name, z)
            s.set_trig(trig)
            v, st = s.solve_walks(z["points"], nWalks=int(z["n_walks"]), maxSteps=int(z["max_steps"]),
                                  eps=float(z["eps"]), seed=int(z["seed"]))
            rep = same(v.ravel(), st.ravel(), z["walk_values"], z["walk_steps"])
            sc2, s2 = _solver_for(name)
            s2.set_trig(trig)
            npts, W = SENS_SIZES.get(name, (8, 256))
            pts = sensitivity_points(sc2, name, npts) if name in SENS_SIZES else sc2.points[:npts]
            gv, gs = s2.solve_walks(pts, nWalks=W, maxSteps=sc2.max_steps, eps=sc2.eps, seed=31337)
            pb = O.Problem.from_scenario(sc2, sigma_bar=s2.sigma_bar or 0.0)
            ov, os_ = pb.solve_walks(pts, W, sc2.max_steps, sc2.eps, 31337)
            orc = same(gv.ravel(), gs.ravel(), ov.astype(np.float64), os_)
            print(f"{name:24s} trig={trig:5s} reference replay ({len(z['walk_steps'])} walks): {rep:.4f}   "
                  f"oracle ({npts}x{W}): {orc:.4f}", flush=True)


if __name__ == "__main__":
    main(sys.argv[1:] or ["variable_coefficients", "dcr_dipole", "notebook_dcr", "laplace_square",
                          "poisson_square", "manufactured_polynomial", "wenner_topography"])
