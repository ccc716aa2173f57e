"""compat="fixed" delta tracking's radial sampler (quirks Q4/Q5 corrected; no device).

The reference's ScreenedGreensDistribution2D (solvers/utils.py:154-195) samples the
unit ball's shape for every radius (Q5) under a clipped envelope (Q4). The fixed
sampler draws rho from the exact radial law of the ball's screened Green's function
at the ball's own shape s = R sqrt(sigma_bar):
    p_s(rho) ~ rho [K0(rho s) - K0(s)/I0(s) I0(rho s)],
    F_s(rho) = (1 - t K1(t) - c t I1(t)) / (1 - 1/I0(s)),  t = rho s.
Both libwost's closed-form CDF and the kernels' table sampler (evaluated on the host
by wost_screened_sample_fixed, same table and arithmetic) are checked here against
an independent evaluation with scipy's Bessel functions.
"""
import numpy as np
import pytest

from dcrmontecarlo_amd import _lib

sp = pytest.importorskip("scipy.special")

SHAPES = [0.0, 1e-4, 1e-2, 0.3, 1.0, 1.7, 2.0, 5.0, 13.3, 39.0, 40.0, 41.0, 120.0, 300.0]


def exact_cdf(rho, s):
    rho = np.asarray(rho, np.float64)
    if s == 0.0:
        with np.errstate(divide="ignore", invalid="ignore"):
            return np.where(rho > 0, rho ** 2 * (1 - 2 * np.log(np.where(rho > 0, rho, 1.0))), 0.0)
    t = rho * s
    c = sp.k0(s) / sp.i0(s)
    with np.errstate(all="ignore"):
        tk1 = np.where(t > 0, t * sp.k1(np.where(t > 0, t, 1.0)), 1.0)
    return (1 - tk1 - c * t * sp.i1(t)) / (1 - 1 / sp.i0(s))


def _sample(s, u):
    u = np.ascontiguousarray(u, np.float32)
    ss = np.full(u.shape, s, np.float32)
    out = np.empty_like(u)
    _lib.check(_lib.lib.wost_screened_sample_fixed(_lib.fptr(ss), _lib.fptr(u), u.size, _lib.fptr(out)))
    return out


@pytest.mark.parametrize("s", SHAPES)
def test_closed_form_cdf_matches_scipy(s):
    rho = np.linspace(0, 1, 1001)
    out = np.empty_like(rho)
    _lib.check(_lib.lib.wost_screened_cdf_fixed(s, _lib.dptr(rho), rho.size, _lib.dptr(out)))
    # scipy's own t K1(t) loses ~7 digits at t ~ 1e-4 (1 - t K1 cancels); libwost uses the series
    tol = 1e-6 if s < 1e-3 else 1e-10
    assert np.max(np.abs(out - exact_cdf(rho, s))) < tol
    assert out[0] == 0.0 and out[-1] == 1.0 and np.all(np.diff(out) >= 0)


@pytest.mark.parametrize("s", SHAPES)
def test_table_sampler_quantiles(s):
    """Stratified quantiles u -> rho(u): F_s(rho(u)) == u within 1e-4 everywhere (between
    table rows too), and the draws' mean within 1e-4 of the law's."""
    n = 200_000
    u = (np.arange(n) + 0.5) / n
    rho = _sample(s, u).astype(np.float64)
    assert np.all((rho >= 0) & (rho <= 1)) and np.all(np.diff(rho) >= 0)
    assert np.max(np.abs(exact_cdf(rho, s) - u)) < 1e-4
    grid = np.linspace(0, 1, 20001)
    mean_exact = 1.0 - np.trapezoid(exact_cdf(grid, s), grid)
    assert abs(rho.mean() - mean_exact) < 1e-4


def test_laplace_limit_and_reference_difference():
    """s -> 0: the Laplace law with its Jacobian, mean 4/9 (the reference's Q3 law has
    mean 1/4); large s: the law concentrates like 1/s (the reference's R = 1 shape does
    not shrink with R, Q5)."""
    u = (np.arange(100_000) + 0.5) / 100_000
    assert abs(_sample(0.0, u).mean() - 4.0 / 9.0) < 1e-4
    m40, m400 = _sample(40.0, u).mean(), _sample(400.0, u).mean()
    assert m40 == pytest.approx(10 * m400, rel=1e-4)
