"""libwost.so: the C ABI of include/wost.h loads and exports every declared entry
point, its pure host helpers behave, and without a GPU it fails loudly (no
compute is attempted here)."""
import ctypes

import numpy as np
import pytest

from dcrmontecarlo_amd import _lib


def test_library_exports_every_declared_symbol():
    declared = _lib.declared_symbols()
    assert len(declared) >= 13
    missing = [s for s in declared if not hasattr(_lib.lib, s)]
    assert not missing, missing
    assert _lib.lib.wost_version() == _lib.ABI_VERSION == 6


def test_num_blocks():
    nb = _lib.lib.wost_num_blocks
    assert nb(48, 1_000_000) == 48 * 245
    assert nb(64, 1000) == 64
    assert nb(3, 4096) == 3 and nb(3, 4097) == 6
    assert nb(0, 10) == 0 and nb(5, 0) == 0


def test_struct_layouts():
    assert ctypes.sizeof(_lib.WostFactor) == 36
    assert ctypes.sizeof(_lib.WostTerm) == 12
    assert ctypes.sizeof(_lib.WostPolyline) == 16
    assert ctypes.sizeof(_lib.WostProblem) == 80
    assert ctypes.sizeof(_lib.WostTiming) == 128


def test_fails_loudly_without_a_device():
    if _lib.device_count() > 0:
        pytest.skip("a HIP device is present")
    from dcrmontecarlo_amd import fields as F
    from dcrmontecarlo_amd.geometry import PolyLinesSimple
    from dcrmontecarlo_amd.solvers import WostSolver_2D

    sq = PolyLinesSimple(np.array([[0, 0], [1, 0], [1, 1], [0, 1], [0, 0]], np.float32))
    with pytest.raises(_lib.WostError, match="no HIP device"):
        WostSolver_2D(sq, F.X)
    with pytest.raises(_lib.WostError):
        sq.distance(np.array([0.5, 0.5], np.float32))


def test_invalid_problems_are_rejected_before_device_use():
    from dcrmontecarlo_amd import fields as F
    from dcrmontecarlo_amd.geometry import PolyLinesSimple
    from dcrmontecarlo_amd.solvers import WostSolver_2D

    with pytest.raises(ValueError, match=">= 2 vertices"):
        WostSolver_2D(PolyLinesSimple(np.zeros((1, 2), np.float32)), F.X)
    with pytest.raises(ValueError, match="non-finite"):
        WostSolver_2D(PolyLinesSimple(np.array([[0, 0], [1, np.nan], [1, 1]], np.float32)), F.X, compat="fixed")
    with pytest.raises(ValueError, match="compat"):
        WostSolver_2D(PolyLinesSimple(np.zeros((3, 2), np.float32)), F.X, compat="corrected")
    with pytest.raises(TypeError, match="a field, a number or a callable"):
        WostSolver_2D(PolyLinesSimple(np.zeros((3, 2), np.float32)), "x**2")
