"""Polylines too long to stage in LDS (wost_walk.h GL): the field-specialised kernel
reads them from global memory and gives the bits of the precompiled kernel, which
stages them (up to the CU's 160 KiB). The reference scans any length
(geometry/PolylinesSimple.py:25-49, :134-197), so the build must not refuse them."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _circle(n, r=1.0):
    t = np.linspace(0.0, 2.0 * np.pi, n, dtype=np.float64)
    p = np.stack([r * np.cos(t), r * np.sin(t)], axis=1).astype(np.float32)
    p[-1] = p[0]
    return p


def _pair(make):
    a = make()
    b = make()
    b.set_jit(False)
    return a, b


def test_long_dirichlet_polyline_global_reads(gpu_available):
    from dcrmontecarlo_amd.fields import X, Y
    from dcrmontecarlo_amd.geometry import PolyLinesSimple
    from dcrmontecarlo_amd.solvers import WostSolver_2D

    D = _circle(6001)                       # 48 KB of vertices: above the 40 KiB staging budget
    a, b = _pair(lambda: WostSolver_2D(PolyLinesSimple(D), X**2 - Y**2))
    pts = np.array([[0.1, 0.2], [-0.5, 0.3], [0.0, -0.7]], np.float32)
    v0, s0 = a.solve_walks(pts, nWalks=2048, maxSteps=1000, eps=1e-3, seed=5)
    assert a.last_timing["jit"] == 1
    v1, s1 = b.solve_walks(pts, nWalks=2048, maxSteps=1000, eps=1e-3, seed=5)
    assert b.last_timing["jit"] == 0
    np.testing.assert_array_equal(s0, s1)
    np.testing.assert_array_equal(v0, v1)
    _, st = a.solve(pts, nWalks=100_000, maxSteps=1000, eps=1e-3, seed=6, return_stats=True)
    exact = pts[:, 0].astype(np.float64) ** 2 - pts[:, 1].astype(np.float64) ** 2
    assert np.all(np.abs(st.mean - exact) <= 5 * st.stderr + 3e-3), (st.mean, exact)


def test_long_neumann_polyline_under_fixed_compat(gpu_available):
    """compat="fixed" on a 6000-segment zero-flux line y = 0 across the rectangle
    [0,1] x [-0.5,1] (Dirichlet all round), u = x harmonic with u_y = 0 on it. The
    nearest-crossing queries through the segment tree (field-specialised and
    precompiled kernels) give the bits of the full scans (the specialised kernel
    reading the line from global memory, the precompiled one staging it). A ray
    through a vertex of the line can slip between its two segments in float
    arithmetic; such a walk then ends on the lower Dirichlet side, where u = x holds
    as well, so the exact solution stands."""
    from dcrmontecarlo_amd.fields import X
    from dcrmontecarlo_amd.geometry import PolyLinesSimple
    from dcrmontecarlo_amd.solvers import WostSolver_2D

    n = 6001
    xs = np.linspace(1.0, 0.0, n, dtype=np.float32)
    N = np.stack([xs, np.zeros(n, np.float32)], axis=1)            # y = 0, right to left
    D = np.array([[0, -0.5], [1, -0.5], [1, 1], [0, 1], [0, -0.5]], np.float32)
    a, b = _pair(lambda: WostSolver_2D(PolyLinesSimple(D), X, PolyLinesSimple(N), compat="fixed"))
    pts = np.array([[0.3, 0.5], [0.6, 0.1], [0.8, 0.7]], np.float32)
    v0, s0 = a.solve_walks(pts, nWalks=1024, maxSteps=2000, eps=1e-3, seed=7)
    assert a.last_timing["jit"] == 1
    v1, s1 = b.solve_walks(pts, nWalks=1024, maxSteps=2000, eps=1e-3, seed=7)
    np.testing.assert_array_equal(s0, s1)
    np.testing.assert_array_equal(v0, v1)
    for jit in (True, False):                                      # the scans
        c = WostSolver_2D(PolyLinesSimple(D), X, PolyLinesSimple(N), compat="fixed")
        c.set_jit(jit)
        c.set_segment_tree(-1)
        v2, s2 = c.solve_walks(pts, nWalks=1024, maxSteps=2000, eps=1e-3, seed=7)
        np.testing.assert_array_equal(s0, s2)
        np.testing.assert_array_equal(v0, v2)
    _, st = a.solve(pts, nWalks=50_000, maxSteps=2000, eps=1e-3, seed=8, return_stats=True)
    assert np.all(np.abs(st.mean - pts[:, 0]) <= 5 * st.stderr + 3e-3), (st.mean, pts[:, 0])


def test_history_size_is_checked_before_allocating(gpu_available, monkeypatch):
    from dcrmontecarlo_amd.fields import X
    from dcrmontecarlo_amd.geometry import PolyLinesSimple
    from dcrmontecarlo_amd.solvers import WostSolver_2D

    s = WostSolver_2D(PolyLinesSimple(np.array([[0, 0], [1, 0], [1, 1], [0, 1], [0, 0]], np.float32)), X)
    monkeypatch.setenv("WOST_HISTORY_MAX_BYTES", str(1 << 20))
    with pytest.raises(ValueError, match="return_history"):
        s.solve(np.full((100, 2), 0.5, np.float32), nWalks=1000, maxSteps=1000, return_history=True)


def test_fixed_topography_tree_equals_scan(gpu_available):
    """C5's 10k-segment topography under compat="fixed" (delta tracking, mixed):
    the tree kernel's walks are bitwise those of the full scan."""
    from dcrmontecarlo_amd import scenarios as S

    sc = S.wenner_topography(n_electrodes=16, n_walks=1, n_segments=10_000)
    a = sc.solver(device=0, compat="fixed")
    b = sc.solver(device=0, compat="fixed")
    b.set_segment_tree(-1)
    # the literal C5 fields (sigma_bar 0.5, electrodes ~300 from the Dirichlet sides)
    # would need ~1e4 steps per walk: truncated walks on purpose, for the bit comparison
    for s in (a, b):
        s.set_fixed_step_check(False)
    pts = sc.points[::4]
    v0, s0 = a.solve_walks(pts, nWalks=256, maxSteps=200, eps=sc.eps, seed=3)
    v1, s1 = b.solve_walks(pts, nWalks=256, maxSteps=200, eps=sc.eps, seed=3)
    np.testing.assert_array_equal(s0, s1)
    np.testing.assert_array_equal(v0, v1)
