"""The two-pass scans the field-specialised kernels use for compiled-in Neumann
polylines of 9-65 vertices (wost_jit.cpp; C3's 32-segment circle):

* intersect_polylines_lines -- candidates from one signed line distance per vertex
  (no reciprocal per segment) with a proven slack, then the exact test;
* silhouette_distance_compact -- silhouette vertices marked in a bit mask, squared
  distances only for those;

both bit for bit the one-pass scans (geometry/PolylinesSimple.py:83-102, :134-197
as wost_device.h restates them), on the host build of the device code: the C3
circle, closed zig-zags, open random polylines, collinear and near-parallel rays,
rays through vertices, points on and near the polyline and far away."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


@pytest.fixture(scope="module")
def lib(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("scan") / "libscan_check.so")
    subprocess.run(["/opt/rocm/bin/hipcc", "-O2", "-std=c++17", "-fPIC", "-shared", "--offload-arch=gfx950",
                    "-I" + os.path.join(REPO, "include"), *os.environ.get("WOST_SCAN_CHECK_DEFS", "").split(), "-x", "hip", os.path.join(HERE, "native", "scan_check.cpp"),
                    "-o", out], check=True)
    lb = ctypes.CDLL(out)
    fp = ctypes.POINTER(ctypes.c_float)
    lb.scan_check.argtypes = [fp, ctypes.c_int, fp, fp, fp, ctypes.c_long, ctypes.POINTER(ctypes.c_long)]
    lb.scan_check.restype = ctypes.c_int
    lb.scan_both_check.argtypes = lb.scan_check.argtypes
    lb.scan_both_check.restype = ctypes.c_int
    return lb


def _queries(rng, V, n):
    lo, hi = V.min(0), V.max(0)
    span = hi - lo + 1e-3
    k = n // 4
    a = lo - 0.5 * span + rng.random((k, 2)) * 2.0 * span                      # around the polyline
    i = rng.integers(0, len(V) - 1, n - k)
    t = rng.random(n - k)
    base = V[i] + t[:, None] * (V[i + 1] - V[i])
    b = base + rng.normal(size=(n - k, 2)) * 10.0 ** rng.uniform(-7, 0, (n - k, 1)) * span.max()
    pts = np.concatenate([a, b])
    th = rng.random(n) * 2 * np.pi
    dirs = np.stack([np.cos(th), np.sin(th)], 1) * rng.choice([1.0, 3.0], (n, 1))
    m = (n - k) // 2                                                            # along their segment
    u = V[i[:m] + 1] - V[i[:m]]
    rot = rng.normal(size=m) * 10.0 ** rng.uniform(-9, -2, m)
    c, s = np.cos(rot), np.sin(rot)
    dirs[k:k + m] = np.stack([u[:, 0] * c - u[:, 1] * s, u[:, 0] * s + u[:, 1] * c], 1) * rng.choice([-1, 1], (m, 1))
    j = rng.integers(0, len(V), n // 8)                                          # aimed at vertices
    dirs[-len(j):] = V[j] - pts[-len(j):]
    radii = 10.0 ** rng.uniform(-3, 1, n) * span.max()
    f = lambda x: np.ascontiguousarray(x, np.float32)
    return f(pts), f(dirs), f(radii)


def _c3_circle():
    from dcrmontecarlo_amd import scenarios as S

    return S.variable_coefficients(n_points=1, n_walks=1).neumann


def _shapes():
    rng = np.random.default_rng(0)
    th = np.linspace(0, 2 * np.pi, 17)
    zig = np.stack([np.cos(th) * (1 + 0.4 * (np.arange(17) % 2)), np.sin(th) * (1 + 0.4 * (np.arange(17) % 2))], 1)
    zig[-1] = zig[0]
    return {"c3_circle": _c3_circle(), "zigzag17": zig * 3.0,
            "open9": np.cumsum(rng.normal(size=(9, 2)), 0) + 50.0,
            "open65": np.cumsum(rng.normal(size=(65, 2)), 0) * 0.01,
            "flat65": np.stack([np.linspace(-1e3, 1e3, 65), np.zeros(65)], 1)}


@pytest.mark.parametrize("shape", list(_shapes()))
def test_two_pass_compiled_scans_match_one_pass(lib, shape):
    V = np.ascontiguousarray(_shapes()[shape], np.float32)
    rng = np.random.default_rng(len(V))
    pts, dirs, radii = _queries(rng, V.astype(np.float64), 80_000)
    out = (ctypes.c_long * 4)()
    p = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))
    assert lib.scan_check(p(V), len(V), p(pts), p(dirs), p(radii), len(pts), out) == 0
    assert out[0] == 0 and out[1] == 0, list(out)
    assert out[2] > 1000, list(out)                       # the ray query exercised
    assert out[3] > 1000 or shape == "flat65", list(out)  # (a straight line has no silhouette)


def _long_shapes():
    from dcrmontecarlo_amd import scenarios as S

    rng = np.random.default_rng(1)
    th = np.linspace(0, 2 * np.pi, 2001)
    wig = np.stack([np.cos(th) * (1 + 0.05 * np.sin(37 * th)), np.sin(th) * (1 + 0.05 * np.sin(37 * th))], 1) * 40.0
    return {"topography10k": S.topography(10_000), "wiggly_circle2001": wig,
            "random_walk1003": np.cumsum(rng.normal(size=(1003, 2)), 0),
            "flat66": np.stack([np.linspace(-1e3, 1e3, 66), np.zeros(66)], 1),
            "zigzag67": np.stack([np.arange(67.0), (np.arange(67) % 2) * 3.0], 1)}


@pytest.mark.parametrize("shape", list(_long_shapes()))
def test_fused_bruteforce_scan_matches_both_scans(lib, shape):
    """neumann_scan_both (the brute-force kernels' one pass over a long polyline, batches of
    eight vertices, the last one partial) returns silhouette_distance's and
    intersect_polylines<false>'s bits."""
    V = np.ascontiguousarray(_long_shapes()[shape], np.float32)
    rng = np.random.default_rng(len(V) + 7)
    pts, dirs, radii = _queries(rng, V.astype(np.float64), 4000 if len(V) > 5000 else 20_000)
    out = (ctypes.c_long * 4)()
    p = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))
    assert lib.scan_both_check(p(V), len(V), p(pts), p(dirs), p(radii), len(pts), out) == 0
    assert out[0] == 0 and out[1] == 0, list(out)
    assert out[2] > 200, list(out)
    assert out[3] > 200 or shape == "flat66", list(out)
