"""compat="fixed": the Walk-on-Stars estimator with the reference's quirks
corrected (Q1-Q5, Q7, Q12, Q13; wost_walk.h FIX).

The reference has no such mode, so there is nothing to be bit-identical to:
these tests pin it by exact solutions instead. Each problem is chosen so that a
quirk the fixed mode corrects would bias the reference mode:
* Poisson with a curved source (u = x^4 + y^2): Q3, the missing Jacobian of
  the Green's radial density, biases compat="reference";
* mixed Dirichlet / Neumann (u = x on the unit square, zero flux on top):
  Q1/Q2, the segment-parameter ray time and the rotated hemisphere, bias it;
* Laplace (u = x^2 - y^2) and eps >= 1 (Q12).
* delta tracking (the reference's polynomial manufactured solution, and a mixed
  problem with zero flux on one side): Q4/Q5, the clipped unit-ball screened law
  without its Jacobian, biases compat="reference".
The fixed mode must agree with the exact solution within Monte-Carlo error and
run bit-identically in the specialised and precompiled kernels.
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


# ---------------------------------------------------------------- delta tracking (Q4/Q5)
def _poly_problem():
    """The reference's polynomial manufactured solution (tests/testWoStCorrectness.py:81-142):
    u = (1-x^2)(1-y^2) on [-1,1]^2, diffusion alpha = 2 + x/2 + y/2, absorption
    sigma = 2 + xy, f = -div(alpha grad u) + sigma u."""
    from dcrmontecarlo_amd.fields import X, Y

    u = (1 - X**2) * (1 - Y**2)
    alpha = 2.0 + 0.5 * X + 0.5 * Y
    sigma = 2.0 + X * Y
    lap = -2.0 * (2.0 - X**2 - Y**2)
    grad_dot = -X * (1 - Y**2) - Y * (1 - X**2)       # grad(alpha) . grad(u)
    f = -(alpha * lap + grad_dot) + sigma * u
    pts = np.array([[-0.5, 0.2], [0.0, 0.0], [0.6, -0.3], [0.3, 0.7], [-0.7, -0.6]], np.float32)
    exact = (1 - pts[:, 0].astype(np.float64) ** 2) * (1 - pts[:, 1].astype(np.float64) ** 2)
    return u, alpha, sigma, f, pts, exact


def _mixed_problem():
    """Unit square, Dirichlet on the left, bottom and right sides, zero-flux Neumann top:
    u = 1 + x^2 + (1+x)(2y - y^2)/2 has u_y = 0 at y = 1; alpha = 1 + x/2, sigma = 1 + y.
    The source is nonzero up to the Neumann side, so the walks' source samples on that
    boundary (the half-ball) carry weight."""
    from dcrmontecarlo_amd.fields import X, Y

    u = 1.0 + X**2 + 0.5 * (1.0 + X) * (2.0 * Y - Y**2)
    alpha = 1.0 + 0.5 * X
    sigma = 1.0 + Y
    lap = 1.0 - X                                        # u_xx + u_yy = 2 - (1 + x)
    grad_dot = 0.5 * (2.0 * X + 0.5 * (2.0 * Y - Y**2))  # (1/2, 0) . grad(u)
    f = -(alpha * lap + grad_dot) + sigma * u
    pts = np.array([[0.3, 0.5], [0.5, 0.9], [0.7, 0.97], [0.2, 0.2], [0.5, 0.99]], np.float32)
    x, y = pts[:, 0].astype(np.float64), pts[:, 1].astype(np.float64)
    exact = 1 + x ** 2 + 0.5 * (1 + x) * (2 * y - y ** 2)
    return u, alpha, sigma, f, pts, exact


def test_fixed_delta_tracking_is_unbiased(gpu_available):
    """Delta tracking with the corrected screened sampler (Q4/Q5) agrees with the exact
    solution; the reference mode's clipped unit-ball law without the Jacobian does not."""
    u, alpha, sigma, f, pts, exact = _poly_problem()
    fixed = _solver(SQUARE1, u, f=f, sigma=sigma, alpha=alpha, compat="fixed")
    assert fixed.use_delta_tracking and fixed.sigma_bar > 0
    _, st = fixed.solve(pts, nWalks=400_000, maxSteps=2000, eps=1e-4, seed=21, return_stats=True)
    assert np.all(np.abs(st.mean - exact) <= 5 * st.stderr + 2e-3), (st.mean, exact, st.stderr)
    ref = _solver(SQUARE1, u, f=f, sigma=sigma, alpha=alpha)
    _, sr = ref.solve(pts, nWalks=400_000, maxSteps=2000, eps=1e-4, seed=21, return_stats=True)
    assert np.max(np.abs(_z(sr, exact))) > 10, "the reference-mode Q4/Q5 bias should be visible here"


def test_fixed_delta_signed_collision_weights(gpu_available):
    """sigma_bar below max sigma' (here 1.0 against ~2.9): the fixed mode keeps the
    collision weight 1 - sigma'/sigma_bar signed and stays unbiased."""
    u, alpha, sigma, f, pts, exact = _poly_problem()
    s = _solver(SQUARE1, u, f=f, sigma=sigma, alpha=alpha, compat="fixed", sigma_bar=1.0)
    assert s.sigma_bar == 1.0
    _, st = s.solve(pts, nWalks=400_000, maxSteps=2000, eps=1e-4, seed=22, return_stats=True)
    assert np.all(np.abs(st.mean - exact) <= 5 * st.stderr + 2e-3), (st.mean, exact, st.stderr)


def test_fixed_mixed_delta_tracking_is_unbiased(gpu_available):
    """Delta tracking with a Neumann side: nearest ray crossings (Q1), inward hemispheres
    for the step and the source sample (Q2, Q13), collisions outside the star-shaped
    region ending the walk, the corrected sampler (Q4/Q5)."""
    u, alpha, sigma, f, pts, exact = _mixed_problem()
    fixed = _solver(UNIT_U, u, UNIT_TOP, f=f, sigma=sigma, alpha=alpha, compat="fixed")
    _, st = fixed.solve(pts, nWalks=400_000, maxSteps=4000, eps=1e-4, seed=23, return_stats=True)
    assert np.all(np.abs(st.mean - exact) <= 5 * st.stderr + 2e-3), (st.mean, exact, st.stderr)


def test_fixed_mixed_poisson_source_on_the_neumann_side(gpu_available):
    """Poisson with a Neumann side and a source reaching it: on a Neumann boundary point the
    source sample's direction is uniform on the inward hemisphere (the star-shaped region
    is a half-ball). u = x^3 + 2y^3/3 - y^4/2 on the unit square: u_y = 2y^2 (1 - y) is 0 on
    the top side, -lap u = -(6x + 4y - 6y^2)."""
    from dcrmontecarlo_amd.fields import X, Y

    g = X**3 + (2.0 / 3.0) * Y**3 - 0.5 * Y**4
    f = -(6.0 * X + 4.0 * Y - 6.0 * Y**2)
    pts = np.array([[0.3, 0.5], [0.5, 0.9], [0.7, 0.97], [0.5, 0.99]], np.float32)
    x, y = pts[:, 0].astype(np.float64), pts[:, 1].astype(np.float64)
    exact = x ** 3 + 2 * y ** 3 / 3 - y ** 4 / 2
    s = _solver(UNIT_U, g, UNIT_TOP, f=f, compat="fixed")
    _, st = s.solve(pts, nWalks=400_000, maxSteps=4000, eps=1e-4, seed=24, return_stats=True)
    assert np.all(np.abs(st.mean - exact) <= 5 * st.stderr + 2e-3), (st.mean, exact, st.stderr)


@pytest.mark.parametrize("case", ["delta", "mixed_delta"])
def test_fixed_delta_kernels_are_deterministic_and_agree(gpu_available, case):
    u, alpha, sigma, f, pts, _ = _poly_problem() if case == "delta" else _mixed_problem()
    geo = (SQUARE1, None) if case == "delta" else (UNIT_U, UNIT_TOP)
    mk = lambda: _solver(geo[0], u, geo[1], f=f, sigma=sigma, alpha=alpha, compat="fixed")
    a = mk()
    v0, s0 = a.solve_walks(pts, nWalks=8192, maxSteps=2000, eps=1e-4, seed=11)
    v1, s1 = a.solve_walks(pts, nWalks=8192, maxSteps=2000, eps=1e-4, seed=11)
    assert a.last_timing["jit"] == 1
    np.testing.assert_array_equal(v0, v1)
    b = mk()
    b.set_jit(False)
    v2, s2 = b.solve_walks(pts, nWalks=8192, maxSteps=2000, eps=1e-4, seed=11)
    assert b.last_timing["jit"] == 0
    np.testing.assert_array_equal(s0, s2)
    np.testing.assert_array_equal(v0, v2)


def test_fixed_delta_refuses_walks_that_would_all_be_truncated(gpu_available):
    """on the DCR configurations the corrected screened law moves a
    walk ~2/sqrt(sigma_bar) = 0.6 per collision, ~100 from the Dirichlet box: every walk
    would end at maxSteps. compat="fixed" refuses such solves (ValueError naming the
    estimate) in every entry point; with the check off the truncation is plain to see;
    with enough steps for the estimate the solve runs."""
    from dcrmontecarlo_amd import scenarios as S

    sc = S.dcr_dipole(n_electrodes=8, n_walks=1)
    s = sc.solver(device=0, compat="fixed")
    assert s.sigma_bar == pytest.approx(10.0)
    for call in (lambda: s.solve(sc.points, nWalks=256, maxSteps=sc.max_steps, eps=sc.eps, seed=1),
                 lambda: s.solve_walks(sc.points, nWalks=256, maxSteps=sc.max_steps, eps=sc.eps, seed=1),
                 lambda: s.solve_range(sc.points, 4096, 0, 4096, sc.max_steps, sc.eps, 1)):
        with pytest.raises(ValueError, match="truncate"):
            call()
    s.set_fixed_step_check(False)
    _, st = s.solve_walks(sc.points, nWalks=256, maxSteps=sc.max_steps, eps=sc.eps, seed=1)
    assert np.mean(st == sc.max_steps) > 0.99          # what the check prevents
    # the reference mode on the same problem terminates (the ~76 steps of its rescaled law)
    r = sc.solver(device=0)
    _, sr = r.solve_walks(sc.points, nWalks=256, maxSteps=sc.max_steps, eps=sc.eps, seed=1)
    assert np.mean(sr < sc.max_steps) > 0.99
