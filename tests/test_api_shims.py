"""The reference's import paths and small PolyLinesSimple helpers (host only, no device).

* ``solvers.WoStSolver``, ``geometry.PolylinesSimple``, ``geometry.Polylines`` and
  ``utils.torch_smooth_circle`` resolve to the MI355X package (a
  reference scenario script runs without editing its imports);
* ``funcToPolyline`` hands ``func`` a float32 torch tensor like the reference
  (geometry/PolylinesSimple.py:226-240) and keeps quirk Q11 (x starts at 0);
* ``crossProduct2D`` is cross_product_2d_jit (:13-23) with its broadcasting.
"""
import math
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

torch = pytest.importorskip("torch")


def test_reference_import_paths_resolve_to_the_package():
    import dcrmontecarlo_amd as pkg
    from geometry.Polylines import PolyLines
    from geometry.PolylinesSimple import PolyLinesSimple
    from solvers.WoStSolver import WostSolver_2D

    assert WostSolver_2D is pkg.WostSolver_2D
    assert PolyLinesSimple is pkg.PolyLinesSimple
    assert PolyLines is pkg.PolyLines
    assert issubclass(PolyLinesSimple, PolyLines)


def test_torch_smooth_circle_shim_matches_formula_and_traces():
    from dcrmontecarlo_amd import fields as F
    from dcrmontecarlo_amd import trace
    from utils import torch_smooth_circle

    c = torch.tensor([-20, -30])
    for p in ([-20.0, -25.0], [-5.0, -30.0], [-20.0, -40.05], [0.0, 0.0]):
        pt = torch.tensor(p)
        z = -100.0 * (math.hypot(p[0] + 20, p[1] + 30) - 10)
        want = 1.0 / (1.0 + math.exp(-z)) if z > -700 else 0.0
        assert float(torch_smooth_circle(pt, c, 10)) == pytest.approx(want, abs=1e-6)
    # tests/testGeophysicalScenario.py:35-55 written with the shim traces to the scenario's field
    fld = trace.trace(lambda p: 1e2 + (1e1 - 1e2) * torch_smooth_circle(p, torch.tensor([-20, -30]), 10))
    ref = 1e2 + (1e1 - 1e2) * F.smooth_circle((-20.0, -30.0), 10.0)
    pts = np.array([[-20, -25], [-12, -30], [40, 10]], np.float32)
    for p in pts:
        assert float(fld(p)) == pytest.approx(float(ref(p)), rel=1e-6)


def test_func_to_polyline_passes_a_torch_tensor_and_ignores_x_min():
    from dcrmontecarlo_amd.geometry import PolyLinesSimple

    seen = {}

    def height(x):
        seen["type"] = type(x)
        return 1.0 + 2.0 * torch.sin(x / 37.0)      # torch-only: fails on a numpy array

    poly = PolyLinesSimple.funcToPolyline(height, -50.0, 10.0, 0.5)
    assert seen["type"] is torch.Tensor
    ref_x = torch.arange(0, 10.0, 0.5)                # what the reference samples (x_min ignored, Q11)
    assert isinstance(poly.points, torch.Tensor) and poly.points.dtype == torch.float32
    assert torch.equal(poly.points[:, 0], ref_x)
    assert torch.equal(poly.points[:, 1], 1.0 + 2.0 * torch.sin(ref_x / 37.0))
    assert len(poly) == 20


def test_func_to_polyline_accepts_numpy_results():
    from dcrmontecarlo_amd.geometry import PolyLinesSimple

    poly = PolyLinesSimple.funcToPolyline(lambda x: np.zeros(len(x), np.float64), 0.0, 1.0, 0.25)
    assert poly.points.shape == (4, 2)
    assert float(poly.points[:, 1].abs().max()) == 0.0


def test_cross_product_2d_broadcasts_like_the_reference():
    from dcrmontecarlo_amd.geometry import PolyLinesSimple

    poly = PolyLinesSimple(np.array([[0, 0], [1, 0]], np.float32))
    a = torch.tensor([[1.0, 2.0], [3.0, -4.0], [0.5, 0.25]])
    b = torch.tensor([2.0, 5.0])
    got = poly.crossProduct2D(a, b)
    want = a[:, 0] * b[1] - a[:, 1] * b[0]              # cross_product_2d_jit (:13-23)
    assert isinstance(got, torch.Tensor)
    assert torch.equal(got, want)
    single = poly.crossProduct2D(np.array([1.0, 0.0], np.float32), np.array([0.0, 1.0], np.float32))
    assert np.asarray(single).ravel()[0] == 1.0


def test_utils_autograd_helpers_and_plot_stubs():
    """The root utils shim's host helpers (reference utils.py:11-120): gradient,
    Laplacian with its +1e-8 offset, grid min/max; the plotting functions (out of
    scope) raise NotImplementedError instead of failing on import."""
    import utils

    p = torch.tensor([1.0, 2.0])
    g = utils.torchGradient(lambda x: x[0] ** 2 + 3 * x[1], p)
    assert g.tolist() == [2.0, 3.0]
    assert float(utils.torchLaplacian(lambda x: x[0] ** 4 + x[1] ** 4, p)) == pytest.approx(60.0)
    # a linear function: its gradient has no graph, the second derivative raises and
    # the 1e-8 offset comes back (the reference's silent fallback)
    assert float(utils.torchLaplacian(lambda x: x[0] + 2 * x[1], p)) == pytest.approx(1e-8, rel=1e-6)
    lo, hi, plo, phi = utils.gridSampleMinMax(lambda x: (x[0] - 0.5) ** 2 + x[1] ** 2, [[0.0, 1.0], [0.0, 1.0]], 11)
    assert lo == pytest.approx(0.0) and hi == pytest.approx(1.25)
    assert plo.tolist() == pytest.approx([0.5, 0.0]) and phi.tolist() == pytest.approx([0.0, 1.0])
    with pytest.raises(ValueError):
        utils.gridSampleMinMax(lambda x: x[0] / 0.0 * 0.0, [[0.0, 1.0]], 5)
    for name in ("plot_walk_history", "plot_multiple_walks", "plot_walk_statistics"):
        with pytest.raises(NotImplementedError):
            getattr(utils, name)({})
