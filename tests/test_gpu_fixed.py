"""compat="fixed": the Walk-on-Stars estimator with the reference's quirks
corrected (Q1-Q3, Q7, Q12, Q13; wost_walk.h FIX).

The reference has no such mode, so there is nothing to be bit-identical to:
these tests pin it by exact solutions instead. Each problem is chosen so that a
quirk the fixed mode corrects would bias the reference mode:
* Poisson with a curved source (u = x^4 + y^2): Q3, the missing Jacobian of
  the Green's radial density, biases compat="reference";
* mixed Dirichlet / Neumann (u = x on the unit square, zero flux on top):
  Q1/Q2, the segment-parameter ray time and the rotated hemisphere, bias it;
* Laplace (u = x^2 - y^2) and eps >= 1 (Q12).
The fixed mode must agree with the exact solution within Monte-Carlo error,
run bit-identically in the specialised and precompiled kernels, and refuse
delta tracking (sigma/alpha), which it does not cover.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _solver(D, g, N=None, f=None, **kw):
    from dcrmontecarlo_amd.geometry import PolyLinesSimple
    from dcrmontecarlo_amd.solvers import WostSolver_2D

    return WostSolver_2D(PolyLinesSimple(D), g, PolyLinesSimple(N) if N is not None else None, source=f, **kw)


SQUARE1 = np.array([[-1, -1], [1, -1], [1, 1], [-1, 1], [-1, -1]], np.float32)
UNIT_U = np.array([[0, 1], [0, 0], [1, 0], [1, 1]], np.float32)      # Dirichlet: left, bottom, right
UNIT_TOP = np.array([[1, 1], [0, 1]], np.float32)                     # Neumann: top


def _z(st, exact):
    return (st.mean - exact) / np.maximum(st.stderr, 1e-12)


def test_fixed_poisson_varying_source_is_unbiased(gpu_available):
    from dcrmontecarlo_amd.fields import X, Y

    # -lap u = f for u = x^4 + y^2; f is not linear, so the radial law of the source
    # sample matters (a linear f averages out over the uniform direction)
    g, f = X**4 + Y**2, -12.0 * X**2 - 2.0
    pts = np.array([[-0.5, 0.2], [0.0, 0.0], [0.6, -0.3], [0.3, 0.7]], np.float32)
    exact = pts[:, 0].astype(np.float64) ** 4 + pts[:, 1].astype(np.float64) ** 2
    fixed = _solver(SQUARE1, g, f=f, compat="fixed")
    _, st = fixed.solve(pts, nWalks=400_000, maxSteps=1000, eps=1e-4, seed=3, return_stats=True)
    assert np.all(np.abs(st.mean - exact) <= 5 * st.stderr + 2e-3), (st.mean, exact, st.stderr)
    ref = _solver(SQUARE1, g, f=f)
    _, sr = ref.solve(pts, nWalks=400_000, maxSteps=1000, eps=1e-4, seed=3, return_stats=True)
    assert np.max(np.abs(_z(sr, exact))) > 10, "the reference-mode Q3 bias should be visible here"


def test_fixed_mixed_neumann_is_unbiased(gpu_available):
    from dcrmontecarlo_amd.fields import X

    pts = np.array([[0.3, 0.5], [0.5, 0.8], [0.7, 0.95], [0.2, 0.2]], np.float32)
    exact = pts[:, 0].astype(np.float64)
    fixed = _solver(UNIT_U, X, UNIT_TOP, compat="fixed")
    _, st = fixed.solve(pts, nWalks=200_000, maxSteps=2000, eps=1e-4, seed=5, return_stats=True)
    assert np.all(np.abs(st.mean - exact) <= 5 * st.stderr + 2e-3), (st.mean, exact, st.stderr)
    ref = _solver(UNIT_U, X, UNIT_TOP)
    _, sr = ref.solve(pts, nWalks=200_000, maxSteps=2000, eps=1e-4, seed=5, return_stats=True)
    # the reference mode is off by many standard errors -- or worse: with Q1 a "hit" may
    # land beyond the Neumann side, walks escape the open top and their radii overflow
    off = ~np.isfinite(sr.mean) | (np.abs(_z(sr, exact)) > 10)
    assert off.any(), "the reference-mode Q1/Q2 bias should be visible here"


def test_fixed_laplace_and_eps_above_one(gpu_available):
    from dcrmontecarlo_amd.fields import X, Y

    sq = np.array([[0, 0], [1, 0], [1, 1], [0, 1], [0, 0]], np.float32)
    pts = np.array([[0.25, 0.5], [0.5, 0.5], [0.8, 0.3]], np.float32)
    exact = pts[:, 0].astype(np.float64) ** 2 - pts[:, 1].astype(np.float64) ** 2
    s = _solver(sq, X**2 - Y**2, compat="fixed")
    _, st = s.solve(pts, nWalks=200_000, maxSteps=1000, eps=1e-4, seed=9, return_stats=True)
    assert np.all(np.abs(st.mean - exact) <= 5 * st.stderr + 1e-3)
    # Q12: the reference never walks when eps >= 1 (dD starts at 1.0); fixed mode stops at the
    # first point only when it is already within eps of the boundary
    _, st2 = s.solve(pts, nWalks=64, maxSteps=1000, eps=1.0, seed=9, return_stats=True)
    assert np.all(st2.mean_steps == 0)          # every point is within 1.0 of the square's sides
    big = np.array([[-3, -3], [3, -3], [3, 3], [-3, 3], [-3, -3]], np.float32)
    s3 = _solver(big, X**2 - Y**2, compat="fixed")
    _, st3 = s3.solve(np.array([[0.0, 0.0]], np.float32), nWalks=1000, maxSteps=1000, eps=1.0, seed=1,
                      return_stats=True)
    assert st3.mean_steps[0] >= 1                # 3 > eps: the fixed walk takes steps
    r3 = _solver(big, X**2 - Y**2)
    _, sr3 = r3.solve(np.array([[0.0, 0.0]], np.float32), nWalks=1000, maxSteps=1000, eps=1.0, seed=1,
                      return_stats=True)
    assert sr3.mean_steps[0] == 0                # the reference's quirk Q12


@pytest.mark.parametrize("case", ["poisson", "mixed_source"])
def test_fixed_kernels_are_deterministic_and_agree(gpu_available, case):
    from dcrmontecarlo_amd.fields import X, Y

    if case == "poisson":
        mk = lambda: _solver(SQUARE1, X**3 + Y**2, f=-6.0 * X - 2.0, compat="fixed")
        pts = np.array([[0.1, 0.2], [-0.4, 0.5]], np.float32)
    else:
        mk = lambda: _solver(UNIT_U, X, UNIT_TOP, f=1.0 + X * Y, compat="fixed")
        pts = np.array([[0.3, 0.9], [0.6, 0.5]], np.float32)
    a = mk()
    v0, s0 = a.solve_walks(pts, nWalks=8192, maxSteps=1000, eps=1e-4, seed=11)
    v1, s1 = a.solve_walks(pts, nWalks=8192, maxSteps=1000, eps=1e-4, seed=11)
    assert a.last_timing["jit"] == 1
    np.testing.assert_array_equal(v0, v1)
    b = mk()
    b.set_jit(False)
    v2, s2 = b.solve_walks(pts, nWalks=8192, maxSteps=1000, eps=1e-4, seed=11)
    assert b.last_timing["jit"] == 0
    np.testing.assert_array_equal(s0, s2)
    np.testing.assert_array_equal(v0, v2)


def test_fixed_refuses_delta_tracking(gpu_available):
    from dcrmontecarlo_amd.fields import X

    with pytest.raises(NotImplementedError):
        _solver(SQUARE1, X, f=1.0, sigma=1.0, compat="fixed")
