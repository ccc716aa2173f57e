#!/usr/bin/env python3
"""Record C5 walks on the GPU (return_history) and save every step's point and its
Dirichlet / Neumann distances, for host-side studies of the segment-tree queries at
the positions the walks actually visit. Output: gpurun_out/c5_paths.npz."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    from dcrmontecarlo_amd import scenarios as S

    sc = S.wenner_topography(n_electrodes=256, n_walks=16)
    s = sc.solver(device=0)
    pts = sc.points[::8]
    u, hist = s.solve(pts, nWalks=16, maxSteps=sc.max_steps, eps=sc.eps, seed=5, return_history=True)
    P, DD, DN, E = [], [], [], []
    for i in range(len(pts)):
        for w in hist[i]:
            for st in w["path"]:
                P.append(np.asarray(st["point"], np.float32))
                DD.append(st["dirichlet_distance"])
                DN.append(st["neumann_distance"])
                E.append(i)
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    np.savez_compressed(os.path.join(REPO, "gpurun_out", "c5_paths.npz"), points=np.array(P, np.float32),
                        dd=np.array(DD, np.float32), dn=np.array(DN, np.float32), electrode=np.array(E, np.int32))
    print("steps recorded:", len(P))


if __name__ == "__main__":
    main()
