"""The walk direction's cos/sin (wost_device.h sincos_rn, :230-232) on the host: for every
angle the reference's theta = torch.rand(1) * 2 * pi can take (:226, all 2^24 draws) and
for 2^22 boundary angles theta / 2 + atan2(normal) (:227-228) at the C5 topography's and
the C3 circle's segment angles, sincos_rn equals the C library's double cos/sin rounded to
float32 -- the correctly rounded values, which the reference's torch.cos/torch.sin (MKL)
also return on ~95% of the angles (its own error) -- on all but a handful of angles.
The kernels compute exactly this function, so the device and the oracle (which rounds the
same double results) draw the same directions."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


def segment_phi(V):
    """atan2 of each segment's left normal, as wost_api.hip computes it on the host (the C
    library's atan2f, which torch.atan2 of the reference's 0-d tensors calls)."""
    libm = ctypes.CDLL("libm.so.6")
    libm.atan2f.argtypes = [ctypes.c_float, ctypes.c_float]
    libm.atan2f.restype = ctypes.c_float
    V = np.asarray(V, np.float32)
    u = V[1:] - V[:-1]
    ln = np.sqrt(u[:, 0] * u[:, 0] + u[:, 1] * u[:, 1])
    return np.array([libm.atan2f(float(ex), float(-ey)) for ex, ey in zip(u[:, 0] / ln, u[:, 1] / ln)], np.float32)


@pytest.fixture(scope="module")
def trig_lib(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("trig") / "libtrig_check.so")
    subprocess.run(["/opt/rocm/bin/hipcc", "-O2", "-std=c++17", "-fPIC", "-shared", "--offload-arch=gfx950",
                    "-ffp-contract=off", "-I" + os.path.join(REPO, "include"), "-x", "hip",
                    os.path.join(HERE, "native", "trig_check.cpp"), "-o", out], check=True)
    lib = ctypes.CDLL(out)
    lib.trig_check.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_int, ctypes.c_long,
                               ctypes.POINTER(ctypes.c_long)]
    return lib


def test_walk_direction_is_correctly_rounded(trig_lib):
    from dcrmontecarlo_amd import scenarios as S

    phi = np.concatenate([segment_phi(S.topography(10_000)),
                          segment_phi(S.variable_coefficients(n_points=1, n_walks=1).neumann)]).astype(np.float32)
    c = (ctypes.c_long * 5)()
    assert trig_lib.trig_check(phi.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), len(phi), 1 << 22, c) == 0
    n, bad_s, bad_c, libm_s, libm_c = list(c)
    assert n == (1 << 24) + (1 << 22)
    assert bad_s <= 2 and bad_c <= 2, (bad_s, bad_c)
    print(f"sincos_rn != rounded double: sin {bad_s}, cos {bad_c} of {n}; "
          f"the C library's sinf/cosf: {libm_s / n:.4f}, {libm_c / n:.4f}")
