"""WostSolver_2D built from the reference's kind of Python callables, on the device.

* Traced callables (exact): the solver built from the reference-style
  callables of tests/test_trace.py walks like the solver built from the
  hand-written scenario fields -- the same per-walk step counts and values
  (floors as in test_gpu_parity.test_device_matches_oracle, since a traced
  field may round its constants differently from the hand-written one).
* Tabulated callables (WOST_FK_GRID, approximate): the device interpolation
  equals the oracle's independent restatement, walks agree with the oracle
  walk for walk, the field-specialised and precompiled kernels are
  bit-identical, and on a smooth scenario the tabulated solve agrees with the
  exact-field solve within Monte-Carlo error.
"""
import numpy as np
import pytest

from test_trace import CALLABLES

pytestmark = pytest.mark.gpu

FLOOR = {"laplace_square": 0.99, "manufactured_polynomial": 0.99, "poisson_square": 0.99,
         "variable_coefficients": 0.97, "dcr_dipole": 0.99, "notebook_dcr": 0.99}


def _solvers(name, **kw):
    from dcrmontecarlo_amd import scenarios as S
    from dcrmontecarlo_amd.geometry import PolyLinesSimple
    from dcrmontecarlo_amd.solvers import WostSolver_2D

    sc = S.ALL[name]()
    cb = CALLABLES[name]
    D = PolyLinesSimple(sc.dirichlet)
    N = PolyLinesSimple(sc.neumann) if sc.neumann is not None else None
    ref = WostSolver_2D(D, sc.g, N, source=sc.f, sigma=sc.sigma, alpha=sc.alpha)
    cal = WostSolver_2D(D, cb.get("g"), N, source=cb.get("f"), sigma=cb.get("sigma"), alpha=cb.get("alpha"), **kw)
    return sc, ref, cal


@pytest.mark.parametrize("name", sorted(CALLABLES))
def test_traced_callables_walk_like_scenario_fields(gpu_available, name):
    sc, ref, cal = _solvers(name)
    assert all(c.how in ("traced", "constant") for c in cal.field_conversions.values()), cal.field_conversions
    assert cal.use_delta_tracking == ref.use_delta_tracking
    if ref.sigma_bar is not None:
        assert cal.sigma_bar == pytest.approx(ref.sigma_bar, rel=1e-5)
    pts = sc.points[:4]
    W = 4096
    v0, s0 = ref.solve_walks(pts, nWalks=W, maxSteps=sc.max_steps, eps=sc.eps, seed=19)
    v1, s1 = cal.solve_walks(pts, nWalks=W, maxSteps=sc.max_steps, eps=sc.eps, seed=19)
    assert cal.last_timing["jit"] == 1
    scale = max(float(np.abs(v0).max()), 1e-30)
    same = (s0 == s1) & (np.abs(v1 - v0) <= 1e-3 * np.abs(v0) + 1e-5 * scale)
    assert same.mean() >= FLOOR[name], same.mean()


def _tabulated_solver(name, resolution=257):
    return _solvers(name, trace_callables=False, grid_resolution=resolution)


def test_tabulated_fields_match_oracle(gpu_available):
    """FK_GRID on the device (values, gradient, Laplacian through sigma') vs the
    oracle's double-precision Hermite-form restatement of the same grid."""
    from oracle import oracle as O

    with pytest.warns(RuntimeWarning, match="tabulating"):
        sc, ref, cal = _tabulated_solver("variable_coefficients")
    assert all(c.how == "tabulated" for c in cal.field_conversions.values())
    rng = np.random.default_rng(4)
    P = rng.uniform(-1.6, 1.6, (512, 2)).astype(np.float32)   # includes points just outside the domain
    for which in ("g", "f", "sigma", "alpha"):
        got = cal.eval_field(which, P)[:, 0]
        fld = {"g": cal.boundaryDirichlet, "f": cal.source, "sigma": cal.sigma, "alpha": cal.alpha}[which]
        np.testing.assert_allclose(got, O.field_value(fld, P), rtol=2e-5, atol=2e-6, err_msg=which)
        np.testing.assert_allclose(got, fld(P), rtol=2e-5, atol=2e-6, err_msg=which)
    pb = O.Problem(sc.dirichlet, sc.neumann, cal.boundaryDirichlet, cal.source, cal.sigma, cal.alpha)
    sp_dev = cal.eval_field("sigma_prime", P)[:, 0]
    np.testing.assert_allclose(sp_dev, pb.sigma_prime(P), rtol=1e-4, atol=1e-5)
    assert cal.sigma_bar == pytest.approx(pb.sigma_bar(), rel=1e-4)


def test_tabulated_walks_match_oracle_and_jit(gpu_available):
    from oracle import oracle as O

    with pytest.warns(RuntimeWarning):
        sc, ref, cal = _tabulated_solver("variable_coefficients")
    pts = sc.points[:4]
    W = 4096
    v1, s1 = cal.solve_walks(pts, nWalks=W, maxSteps=sc.max_steps, eps=sc.eps, seed=23)
    assert cal.last_timing["jit"] == 1
    cal.set_jit(False)
    v0, s0 = cal.solve_walks(pts, nWalks=W, maxSteps=sc.max_steps, eps=sc.eps, seed=23)
    assert np.array_equal(s0, s1) and np.array_equal(v0, v1)
    pb = O.Problem(sc.dirichlet, sc.neumann, cal.boundaryDirichlet, cal.source, cal.sigma, cal.alpha,
                   sigma_bar=cal.sigma_bar)
    ov, os_ = pb.solve_walks(pts, W, sc.max_steps, sc.eps, 23)
    scale = max(float(np.abs(ov).max()), 1e-30)
    same = (os_ == s1.ravel()) & (np.abs(v1.ravel() - ov) <= 1e-3 * np.abs(ov) + 1e-5 * scale)
    assert same.mean() >= 0.97, same.mean()


@pytest.mark.parametrize("name", ["manufactured_polynomial", "variable_coefficients", "poisson_square"])
def test_tabulated_solve_agrees_with_exact_fields(gpu_available, name):
    with pytest.warns(RuntimeWarning):
        sc, ref, cal = _tabulated_solver(name, resolution=513)
    pts = sc.points[:8]
    W = 200_000
    _, a = ref.solve(pts, nWalks=W, maxSteps=sc.max_steps, eps=sc.eps, seed=5, return_stats=True)
    _, b = cal.solve(pts, nWalks=W, maxSteps=sc.max_steps, eps=sc.eps, seed=6, return_stats=True)
    z = (a.mean - b.mean) / np.sqrt(a.stderr**2 + b.stderr**2)
    assert np.all(np.abs(z) < 5), z
