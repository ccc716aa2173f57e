"""The specialised kernels' Dirichlet distance for compiled-in polylines
(wost_device.h poly_distance_const: Markstein division by the constant squared
segment lengths, fmaxf/fminf clamps, no NaN bookkeeping, axis-parallel zero
terms dropped) returns poly_distance's bits (geometry/PolylinesSimple.py:25-49)
on the scenario polylines and random polygons, at random, near-edge,
near-vertex, on-axis and signed-zero points."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from dcrmontecarlo_amd import scenarios as S

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


@pytest.fixture(scope="module")
def lib(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("pd") / "libpolydist_check.so")
    subprocess.run(["/opt/rocm/bin/hipcc", "-O2", "-std=c++17", "-fPIC", "-shared", "--offload-arch=gfx950",
                    "-ffp-contract=off", "-I" + os.path.join(REPO, "include"), "-x", "hip",
                    os.path.join(HERE, "native", "polydist_check.cpp"), "-o", out], check=True)
    lb = ctypes.CDLL(out)
    fp = ctypes.POINTER(ctypes.c_float)
    lb.polydist_check.argtypes = [fp, ctypes.c_int, fp, ctypes.c_long, ctypes.POINTER(ctypes.c_long),
                                  ctypes.POINTER(ctypes.c_int)]
    return lb


def _points(rng, verts, n):
    lo, hi = verts.min(0), verts.max(0)
    span = hi - lo
    k = n // 4
    a = lo - 0.1 * span + rng.random((k, 2)) * 1.2 * span
    i = rng.integers(0, len(verts) - 1, k)
    t = rng.random(k)
    base = verts[i] + t[:, None] * (verts[i + 1] - verts[i])
    b = base + rng.normal(size=(k, 2)) * 10.0 ** rng.uniform(-7, 0, (k, 1)) * span.max()
    c = verts[rng.integers(0, len(verts), k)] + rng.normal(size=(k, 2)) * 10.0 ** rng.uniform(-7, -1, (k, 1))
    d = a[: n - 3 * k].copy()
    d[: len(d) // 2, 0] = verts[rng.integers(0, len(verts), len(d) // 2), 0]   # on a vertex's axis
    d[len(d) // 2:, 1] = 0.0
    extra = np.array([[0.0, 0.0], [-0.0, -0.0], [-0.0, 0.0], [0.0, -0.0]])
    return np.ascontiguousarray(np.concatenate([a, b, c, d, extra]).astype(np.float32))


POLYS = {
    "dcr_box": S.dcr_dipole().dirichlet,
    "variable_coefficients": S.variable_coefficients().dirichlet,
    "notebook_u": S.notebook_dcr().dirichlet,
    "unit_square": S.laplace_square().dirichlet,
    "zero_vertex_box": np.array([[0, 0], [3, 0], [3, 5], [0, 5], [0, 0]], np.float32),
}


@pytest.mark.parametrize("name", sorted(POLYS) + ["random0", "random1"])
def test_poly_distance_const_is_bitwise_poly_distance(lib, name):
    rng = np.random.default_rng(abs(hash(name)) % 2**32)
    if name.startswith("random"):
        ang = np.sort(rng.random(7)) * 2 * np.pi
        rad = rng.uniform(0.5, 3.0, 7)
        verts = np.stack([rad * np.cos(ang), rad * np.sin(ang)], 1) * 10.0 ** rng.uniform(-2, 3)
        verts = np.concatenate([verts, verts[:1]]).astype(np.float32)
    else:
        verts = np.ascontiguousarray(POLYS[name], np.float32)
    pts = _points(rng, verts.astype(np.float64), 200_000)
    bad = ctypes.c_long(-1)
    nm = ctypes.c_int(0)
    p = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))
    assert lib.polydist_check(p(verts), len(verts), p(pts), len(pts), ctypes.byref(bad), ctypes.byref(nm)) == 0
    assert bad.value == 0
    if name in ("dcr_box", "variable_coefficients", "random0", "random1"):
        assert nm.value > 0   # the Markstein division is exercised


def test_filtered_ray_test_is_bitwise_ray_test(lib):
    """ray_segment_time_filtered (hardware-reciprocal candidate filter, then the
    exact s and a sign-only t > 0 test) against both IEEE divisions
    (PolylinesSimple.py:104-132), on random, grazing, tiny-t and degenerate cases."""
    rng = np.random.default_rng(7)
    n = 400_000
    a = rng.normal(size=(n, 2)) * 10.0 ** rng.uniform(-3, 3, (n, 1))
    b = a + rng.normal(size=(n, 2)) * 10.0 ** rng.uniform(-6, 2, (n, 1))
    b[: n // 50] = a[: n // 50]                                            # zero-length segments
    q = rng.normal(size=(n, 2)) * 10.0 ** rng.uniform(-3, 3, (n, 1))
    m = n // 4                                                             # rays starting on / near the segment
    t = rng.random(m)
    q[:m] = a[:m] + t[:, None] * (b[:m] - a[:m]) + rng.normal(size=(m, 2)) * 10.0 ** rng.uniform(-40, -3, (m, 1))
    ang = rng.uniform(0, 2 * np.pi, n)
    d = np.stack([np.cos(ang), np.sin(ang)], 1)
    u = b - a
    par = slice(m, 2 * m)                                                  # (nearly) parallel rays
    d[par] = u[par] / np.maximum(np.linalg.norm(u[par], axis=1, keepdims=True), 1e-30)
    d[par] += rng.normal(size=(m, 2)) * 1e-7
    segs = np.ascontiguousarray(np.concatenate([a, b], 1).astype(np.float32))
    rays = np.ascontiguousarray(np.concatenate([q, d], 1).astype(np.float32))
    lib.raytime_check.argtypes = [ctypes.POINTER(ctypes.c_float)] * 2 + [ctypes.c_long] + \
        [ctypes.POINTER(ctypes.c_long)] * 2
    bad, valid = ctypes.c_long(-1), ctypes.c_long(0)
    p = lambda x: x.ctypes.data_as(ctypes.POINTER(ctypes.c_float))
    assert lib.raytime_check(p(segs), p(rays), n, ctypes.byref(bad), ctypes.byref(valid)) == 0
    assert bad.value == 0
    assert valid.value > n // 20
