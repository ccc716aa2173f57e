"""The walk kernels' screened Green's norm (wost_greens_norm: the device's
table and arithmetic, evaluated on the host) against the reference's
screenedGreensNorm2D values (tests/golden/greens.npz, solvers/utils.py:29-44)
and against the double-precision formula over the whole table range."""
import ctypes

import numpy as np

from conftest import golden
from dcrmontecarlo_amd import _lib


def _gnorm(sigma_bar, r):
    r = np.ascontiguousarray(r, dtype=np.float32)
    out = np.empty_like(r)
    _lib.check(_lib.lib.wost_greens_norm(float(sigma_bar), _lib.fptr(r), r.size, _lib.fptr(out)), "wost_greens_norm")
    return out


def test_greens_norm_matches_reference_golden():
    z = golden("greens.npz")
    for i, sb in enumerate(z["sigma_bar"]):
        got = _gnorm(sb, z["R"]).astype(np.float64)
        np.testing.assert_allclose(got, z["screened_norm"][i], rtol=4e-7, atol=0)


def test_greens_norm_table_range_and_tail():
    for sb in (0.5, 2.40625, 10.0, 137.0):
        s = np.sqrt(sb)
        x = np.concatenate([np.linspace(1e-4, 21.5, 20001), [25.0, 40.0, 300.0, 1e4]])
        r = (x / s).astype(np.float32)
        xd = r.astype(np.float64) * np.float64(np.float32(s))
        with np.errstate(over="ignore"):
            exact = (1.0 - 1.0 / np.i0(xd)) / sb
        got = _gnorm(sb, r).astype(np.float64)
        np.testing.assert_allclose(got, exact, rtol=4e-7, atol=0)
        # beyond the table G_norm is 1/sigma_bar exactly, as float32 1 - 1/I0 rounds to 1
        big = xd >= 256 / 12
        assert np.all(got[big] == np.float32(1.0 / sb))


def test_greens_norm_rejects_bad_arguments():
    r = np.ones(2, np.float32)
    out = np.empty(2, np.float32)
    assert _lib.lib.wost_greens_norm(0.0, _lib.fptr(r), 2, _lib.fptr(out)) == _lib.WOST_ERR_INVALID_ARG
    assert _lib.lib.wost_greens_norm(1.0, None, 2, None) == _lib.WOST_ERR_INVALID_ARG
