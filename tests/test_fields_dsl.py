"""The coefficient-field DSL (dcrmontecarlo_amd.fields): algebra, encoding, host evaluation."""
import math

import numpy as np
import pytest

from dcrmontecarlo_amd import fields as F
from dcrmontecarlo_amd.fields import X, Y


def test_polynomial_algebra_merges_terms():
    f = (1 - X**2) * (1 - Y**2)
    assert f.polynomial() == {(0, 0): 1.0, (2, 0): -1.0, (0, 2): -1.0, (2, 2): 1.0}
    assert (X - X).terms == []
    assert (2 * X + 3 * X).polynomial() == {(1, 0): 5.0}
    p = np.array([[0.3, -0.7], [1.5, 2.0]], np.float32)
    np.testing.assert_allclose(f(p), (1 - p[:, 0] ** 2) * (1 - p[:, 1] ** 2), rtol=1e-6)


def test_exp_of_quadratic_is_centred():
    g = F.exp(-((X + 10) ** 2 + Y**2) / 0.5)
    (coef, first, n), = g.pack()[0]
    kind, p = g.pack()[1][0]
    assert kind == F.FK_EXP_QUAD and n == 1 and coef == 1.0
    assert p[0] == pytest.approx(-10.0) and p[1] == 0.0 and p[2] == -2.0 and p[3] == -2.0
    assert abs(p[5]) < 1e-12 and abs(p[6]) < 1e-12 and abs(p[7]) < 1e-12
    pt = np.array([-10.2, 0.1], np.float32)
    assert g(pt) == pytest.approx(math.exp(-2 * (0.04 + 0.01)), rel=1e-6)


def test_gaussian_and_smooth_circle_match_reference_formulas():
    s = 0.5
    g = F.gaussian((10.0, 0.0), s)
    pt = np.array([9.7, 0.2], np.float32)
    assert g(pt) == pytest.approx(math.exp(-((0.3) ** 2 + 0.04) / (2 * s * s)), rel=1e-5)
    c = F.smooth_circle((-20, -30), 10)           # utils.py:123-129
    pt = np.array([-25.0, -22.0], np.float32)
    d = math.hypot(-5.0, 8.0)
    assert c(pt) == pytest.approx(1 / (1 + math.exp(100 * (d - 10))), rel=1e-5)


def test_trig_and_sigmoid_need_linear_arguments():
    assert F.sin(math.pi * X)(np.array([0.5, 0.0])) == pytest.approx(1.0)
    assert F.cos(2 * X + Y + 1)(np.array([0.0, 0.0])) == pytest.approx(math.cos(1.0), rel=1e-6)
    assert F.sigmoid(10000 * Y)(np.array([0.0, 1.0])) == pytest.approx(1.0)
    with pytest.raises(ValueError):
        F.sin(X * Y)
    with pytest.raises(ValueError):
        F.exp(X**3)
    with pytest.raises(TypeError):
        F.as_field(lambda p: p[0])
    with pytest.raises(TypeError):
        X ** 0.5


def test_indicators_are_closed_sets():
    box = F.indicator_box(-2, 2, -2, 2)
    assert box(np.array([2.0, -2.0])) == 1.0 and box(np.array([2.0001, 0.0])) == 0.0
    disk = F.indicator_disk((0, 0), 1.5)
    assert disk(np.array([1.5, 0.0])) == 1.0 and disk(np.array([1.2, 0.91])) == 0.0


def test_detach_flag_and_constants():
    a = F.detach(0.5 + 1.5 * F.exp(-2 * (X**2 + Y**2)))
    assert a.flags & F.FIELD_DETACHED
    assert F.const(3.0).is_constant() and not X.is_constant()
    assert F.const(0.0).terms == []


def test_pack_layout_matches_abi():
    f = 2.0 * X**2 * Y * F.sin(3 * X) + 4.0
    terms, factors = f.pack()
    assert len(terms) == 2
    t0 = terms[0]
    mono = factors[t0[1]]
    assert mono[0] == F.FK_MONO and mono[1][:2] == (2.0, 1.0)
    assert all(len(p) == 8 for _, p in factors)


def test_torch_evaluation_is_differentiable():
    torch = pytest.importorskip("torch")
    f = F.exp(-(X**2 + Y**2)) * F.sin(math.pi * X)
    p = torch.tensor([0.3, -0.4], requires_grad=True)
    v = f(p)
    (g,) = torch.autograd.grad(v, p)
    x, y = 0.3, -0.4
    e = math.exp(-(x * x + y * y))
    assert float(v) == pytest.approx(e * math.sin(math.pi * x), rel=1e-5)
    assert float(g[0]) == pytest.approx(e * (math.pi * math.cos(math.pi * x) - 2 * x * math.sin(math.pi * x)), rel=1e-4)
