"""Round 5 diagnostic: inputs for tools/r05/trig_probe (the walk kernels' trigonometry on
the device vs the host C library, which the reference's 1-element torch ops call).
Writes gpurun_out/r05/trig_in.bin; compare with trig_compare.py."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
from dcrmontecarlo_amd import scenarios as S  # noqa: E402


def inputs(n_theta=1 << 20, seed=5):
    V = S.topography(10_000).astype(np.float32)
    u = V[1:] - V[:-1]
    ln = np.sqrt(u[:, 0] * u[:, 0] + u[:, 1] * u[:, 1])      # float32, as segment_left_normal
    ex, ey = u[:, 0] / ln, u[:, 1] / ln
    nx, ny = -ey, ex
    yx = np.stack([ny, nx], 1).astype(np.float32)
    rng = np.random.default_rng(seed)
    k = rng.integers(0, 1 << 24, n_theta)
    th = (np.float32(1.0 / 16777216.0) * k.astype(np.float32)) * np.float32(2.0)
    th = (th * np.float32(np.pi)).astype(np.float32)               # :226
    phi = np.arctan2(ny.astype(np.float64), nx.astype(np.float64)).astype(np.float32)
    half = (th[: n_theta // 2] / np.float32(2.0) + phi[rng.integers(0, len(phi), n_theta // 2)]).astype(np.float32)
    th = np.concatenate([th[n_theta // 2:], half]).astype(np.float32)   # :227-228 too
    return yx, th


if __name__ == "__main__":
    out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(REPO, "gpurun_out", "r05", "trig_in.bin")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    yx, th = inputs()
    with open(out, "wb") as f:
        np.array([len(yx), len(th)], np.int32).tofile(f)
        yx.tofile(f)
        th.tofile(f)
    print(out, len(yx), len(th))
