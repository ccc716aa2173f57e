"""Which history field differs from the reference replay (debug aid)."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))
from test_gpu_parity import _solver_for
from conftest import golden
name = sys.argv[1]
z = golden(f"replay_{name}.npz")
sc, s = _solver_for(name, z)
W = int(z["n_walks"]); pts = z["points"]
u, hist = s.solve(pts, nWalks=W, maxSteps=int(z["max_steps"]), eps=float(z["eps"]), seed=int(z["seed"]), return_history=True)
walks = [w for i in range(len(pts)) for w in hist[i]]
off = np.concatenate([[0], np.cumsum(z["walk_steps"])])
rel = lambda a, b: float(np.max(np.abs(a - b) / (1.0 + np.abs(b)))) if np.size(b) else 0.0
for j, w in enumerate(walks[:12]):
    a, b = off[j], off[j + 1]
    P = np.array([np.asarray(st["point"], np.float32) for st in w["path"]]).reshape(-1, 2)
    dd = np.array([st["dirichlet_distance"] for st in w["path"]], np.float32)
    src = [c for c in w["contributions"] if c["type"] == "source"]
    SP = np.array([np.asarray(c["point"], np.float32) for c in src]).reshape(-1, 2)
    SV = np.array([c["contribution"] for c in src], np.float32)
    bnd = w["contributions"][-1]
    print(j, w["steps"], "P", rel(P, z["path_points"][a:b]), "dd", rel(dd, z["path_dd"][a:b]),
          "SP", rel(SP, z["src_points"][a:b]), "SV", rel(SV, z["src_values"][a:b]),
          "bnd", float(bnd["contribution"]), float(z["boundary_values"][j]), "val", w["value"], float(z["walk_values"][j]))
    if j < 2 and len(SV):
        print("   SV ours", SV[:4], "ref", z["src_values"][a:a + 4])
        print("   SP ours", SP[:2].tolist(), "ref", z["src_points"][a:a + 2].tolist())
