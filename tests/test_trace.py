"""Reference-style Python callables -> device fields (dcrmontecarlo_amd.trace).

The callables below are written in the reference's calling convention --
one float32 point tensor in, a float / 0-d tensor out -- with the constructs
its scenario callables use: float() and torch.tensor() re-wrapping, torch
exp/sin/cos/sigmoid, a norm-based smooth circle (utils.py:123-129), and
if-branches on the point (tests/testWostWithSource.py:51-56,
tests/testWostVariableCoefficients.py:74-84). Each traced field is pinned
against the reference's own evaluations of the original callables
(tests/golden/fields_*.npz, tools/gen_fixtures.py), and through the CPU
oracle against the reference's sigma' and sigma_bar.
"""
import math
import warnings

import numpy as np
import pytest
import torch

from conftest import golden
from dcrmontecarlo_amd import fields as F
from dcrmontecarlo_amd import trace as T


def _circle_step(pt, centre, radius):           # the smooth circle of utils.py:123-129
    return (-100 * ((pt - centre).norm() - radius)).sigmoid()


def dcr_source(pt):
    x, y = pt[0], pt[1]
    w = 0.5
    a = 1.0 / (2 * torch.pi * w**2)
    plus = a * torch.exp(-((x + 10.0) ** 2 + y**2) / (2 * w**2))
    minus = -a * torch.exp(-((x - 10.0) ** 2 + y**2) / (2 * w**2))
    return float(plus - minus)                   # both electrodes inject (quirk Q10)


def dcr_alpha(pt):
    bg = 1e2
    return (bg + (1e1 - bg) * _circle_step(pt, torch.tensor([-20, -30]), 10)
            + (1e3 - bg) * _circle_step(pt, torch.tensor([25, -40]), 10))


def nb_alpha(pt):
    bg = 1e-2
    return (bg + (1e-1 - bg) * _circle_step(pt, torch.tensor([-120, -80]), 60)
            + (1e-3 - bg) * _circle_step(pt, torch.tensor([120, -80]), 60)
            + (1e-8 - bg) * torch.sigmoid(10000 * pt[1]))


def nb_source(pt):
    x, y = pt[0], pt[1]
    w = 5.0
    a = 1.0 / (2 * torch.pi * w**2)
    return float(a * torch.exp(-((x + 200.0) ** 2 + y**2) / (2 * w**2))
                 - a * torch.exp(-((x - 200.0) ** 2 + y**2) / (2 * w**2)))


def vc_alpha(pt):
    x, y = pt[0], pt[1]
    return torch.tensor(0.5 + 1.5 * torch.exp(-2.0 * (x**2 + y**2)))      # detached -> sigma/alpha (Q9)


def vc_sigma(pt):
    x, y = pt[0], pt[1]
    return torch.tensor(0.3 + 0.7 * (1 + torch.sin(2 * np.pi * x) * torch.cos(2 * np.pi * y)))


def vc_g(pt):
    return float(torch.sin(np.pi * pt[0]) * torch.sin(np.pi * pt[1]))


def vc_f(pt):
    x, y = pt[0], pt[1]
    rr = x**2 + y**2
    if rr > 1.5**2:
        return 0.0
    return float(torch.exp(-rr) * torch.sin(np.pi * x) * torch.cos(np.pi * y))


def ps_g(pt):
    return float(pt[0] ** 2 + pt[1] ** 2)


def ps_f(pt):
    if pt[0] < -2.0 or pt[0] > 2.0 or pt[1] < -2.0 or pt[1] > 2.0:
        return 0.0
    return -4.0


def mp_alpha(pt):
    return 2.0 + 0.5 * pt[0] + 0.5 * pt[1]


def mp_sigma(pt):
    return pt[0] * pt[1] + 2


def mp_g(pt):
    x, y = pt[0], pt[1]
    return (1 - x**2) * (1 - y**2)


def mp_f(pt):
    x, y = pt[0], pt[1]
    u = (1 - x**2) * (1 - y**2)
    D = 2 + 0.5 * x + 0.5 * y
    return -(D * (-2 * (2 - x**2 - y**2)) + (-x * (1 - y**2) - y * (1 - x**2))) + (2 + x * y) * u


CALLABLES = {
    "dcr_dipole": dict(g=lambda p: 0.0, f=dcr_source, alpha=dcr_alpha),
    "notebook_dcr": dict(g=lambda p: 0.0, f=nb_source, alpha=nb_alpha),
    "variable_coefficients": dict(g=vc_g, f=vc_f, sigma=vc_sigma, alpha=vc_alpha),
    "poisson_square": dict(g=ps_g, f=ps_f),
    "manufactured_polynomial": dict(g=mp_g, f=mp_f, sigma=mp_sigma, alpha=mp_alpha),
    "laplace_square": dict(g=lambda p: p[0] ** 2 - p[1] ** 2),
}


def _bounds(z):
    allp = z["dirichlet"] if "neumann" not in z.files else np.concatenate([z["dirichlet"], z["neumann"]])
    return [[float(allp[:, 0].min()), float(allp[:, 0].max())], [float(allp[:, 1].min()), float(allp[:, 1].max())]]


@pytest.mark.parametrize("name", sorted(CALLABLES))
def test_reference_style_callables_trace_exactly(name):
    """Every scenario callable traces (no tabulation) and the traced field
    reproduces the reference's own evaluation of the original callable."""
    z = golden(f"fields_{name}.npz")
    P = z["points"]
    with warnings.catch_warnings():
        warnings.simplefilter("error", RuntimeWarning)      # a tabulation fallback would warn
        for key, fn in CALLABLES[name].items():
            c = T.field_from_callable(fn, _bounds(z), what=key, is_alpha=(key == "alpha"))
            assert c.how in ("traced", "constant"), (key, c.how, c.detail)
            assert not c.field.is_tabulated()
            if key not in z.files:
                continue
            ref = z[key].astype(np.float64)
            got = np.asarray(c.field(P), np.float64)
            scale = max(np.abs(ref).max(), 1e-30)
            np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-6 * scale, err_msg=f"{name}.{key}")


def test_detachment_follows_the_reference_autograd():
    """torch.tensor(...) re-wrapping detaches alpha (sigma' -> sigma/alpha, Q9);
    a plain torch expression stays differentiable."""
    b = [[-1.5, 1.5], [-1.5, 1.5]]
    assert T.field_from_callable(vc_alpha, b, is_alpha=True).field.flags & F.FIELD_DETACHED
    assert not T.field_from_callable(mp_alpha, b, is_alpha=True).field.flags & F.FIELD_DETACHED
    assert not T.field_from_callable(dcr_alpha, [[-100, 100], [-100, 100]], is_alpha=True).field.flags \
        & F.FIELD_DETACHED
    assert T.alpha_is_detached(lambda p: 1.0, np.zeros((4, 2), np.float32))


@pytest.mark.parametrize("name", ["dcr_dipole", "notebook_dcr", "variable_coefficients", "manufactured_polynomial"])
def test_traced_fields_reproduce_reference_sigma_bar(name):
    """Through the CPU oracle: sigma_bar (50x50 grid of sigma', Q8) and sigma'
    of the traced fields equal the reference's."""
    from oracle import oracle as O

    z = golden(f"fields_{name}.npz")
    b = _bounds(z)
    cv = {k: T.field_from_callable(fn, b, what=k, is_alpha=(k == "alpha")).field for k, fn in CALLABLES[name].items()}
    pb = O.Problem(z["dirichlet"], z["neumann"] if "neumann" in z.files else None, cv.get("g"), cv.get("f"),
                   cv.get("sigma"), cv.get("alpha"))
    assert pb.sigma_bar() == pytest.approx(float(z["sigma_bar"]), rel=1e-4)
    sp = pb.sigma_prime(z["points"]).astype(np.float64)
    ref = z["sigma_prime"]
    fin = np.isfinite(ref)
    np.testing.assert_allclose(sp[fin], ref[fin], rtol=2e-3, atol=1e-5 * np.abs(ref[fin]).max())


def test_branches_become_indicators():
    f = T.trace(ps_f)
    (t,) = f.terms
    assert t.coef == -4.0 and [fc.kind for fc in t.factors] == [F.FK_IND_BOX]
    assert t.factors[0].params[:4] == (-2.0, 2.0, -2.0, 2.0)
    g = T.trace(vc_f)
    assert any(fc.kind == F.FK_IND_DISK for fc in g.terms[0].factors)
    # strict comparisons are exact in float32: x < 1 excludes 1.0 itself
    h = T.trace(lambda p: 1.0 if p[0] < 1.0 else 3.0)
    pts = np.array([[np.nextafter(np.float32(1), np.float32(0)), 0], [1.0, 0], [2.0, 0]], np.float32)
    np.testing.assert_array_equal(h(pts), [1.0, 3.0, 3.0])
    k = T.trace(lambda p: 2.0 if abs(p[1]) <= 0.5 else 0.0)
    np.testing.assert_array_equal(k(np.array([[0, 0.5], [0, -0.5], [0, 0.51]], np.float32)), [2.0, 2.0, 0.0])
    w = T.trace(lambda p: torch.where(p[0] ** 2 + p[1] ** 2 < 1.0, p[0], -p[0]))
    np.testing.assert_allclose(w(np.array([[0.5, 0], [2.0, 0]], np.float32)), [0.5, -2.0])


def test_untraceable_callables_are_tabulated_with_a_warning():
    fn = lambda p: math.exp(-float(p[0]) ** 2) * math.cos(float(p[1]))     # math.* on the point
    b = [[-1.0, 1.0], [-1.0, 1.0]]
    with pytest.warns(RuntimeWarning, match="tabulating"):
        c = T.field_from_callable(fn, b, resolution=129)
    assert c.how == "tabulated" and c.field.is_tabulated()
    rng = np.random.default_rng(0)
    P = rng.uniform(-1, 1, (200, 2)).astype(np.float32)
    exact = np.array([math.exp(-float(x) ** 2) * math.cos(float(y)) for x, y in P])
    np.testing.assert_allclose(c.field(P), exact, atol=2e-5)       # cubic interpolation, h = 1/63


def test_grid_field_numpy_torch_and_oracle_agree():
    """The tabulated factor: numpy (float32), torch (autograd) and the oracle (double,
    own Hermite-form restatement) agree on values; the oracle's analytic gradient
    and Laplacian (used by sigma') agree with finite differences."""
    from oracle import oracle as O

    rng = np.random.default_rng(1)
    vals = rng.standard_normal((9, 13)).astype(np.float32)
    fld = F.tabulated(vals, -1.0, 2.0, 0.25, 0.5)
    P = np.concatenate([rng.uniform([-1.5, 1.5], [2.5, 6.5], (300, 2)),
                        [[-1.0, 2.0], [2.0, 6.0], [0.5, 4.0]]]).astype(np.float32)
    a = fld(P)
    b = O.field_value(fld, P)
    np.testing.assert_allclose(a, b, rtol=1e-5, atol=1e-5)
    # nodes are interpolated exactly
    np.testing.assert_allclose(fld(np.array([[-1.0 + 0.25 * 3, 2.0 + 0.5 * 5]], np.float32)), [vals[5, 3]], rtol=1e-6)
    pt = torch.tensor([0.3, 3.7], requires_grad=True)
    (gr,) = torch.autograd.grad(fld(pt), pt)
    e = 1e-3
    fx = (fld(np.array([0.3 + e, 3.7], np.float32)) - fld(np.array([0.3 - e, 3.7], np.float32))) / (2 * e)
    assert float(gr[0]) == pytest.approx(float(fx), rel=2e-2, abs=2e-2)


def test_tabulated_field_rejects_bad_input():
    with pytest.raises(ValueError):
        F.tabulated(np.zeros((1, 5)), 0, 0, 1, 1)
    with pytest.raises(ValueError):
        F.tabulated(np.zeros((4, 4)), 0, 0, 0.0, 1)
