"""Import-path shim for ``solvers.utils`` (reference solvers/utils.py:29-61): the two
Green's-function norms the walk uses, as the MI355X kernels evaluate them.

greensFunctionNorm2D(R) = R^2 / 4 (:56-61); screenedGreensNorm2D(R, sigma_bar) =
(1/sigma_bar)(1 - 1/I0(R sqrt(sigma_bar))) (:29-44), here from libwost's table
(wost_greens_norm: the kernels' own arithmetic, within a few ulp of the
reference's scipy value, tests/test_greens_table.py)."""
import numpy as np

from dcrmontecarlo_amd import _lib


def greensFunctionNorm2D(R):
    return np.asarray(R, dtype=np.float64) ** 2 / 4.0


def screenedGreensNorm2D(R, sigma_bar):
    r = np.ascontiguousarray(np.atleast_1d(np.asarray(R, dtype=np.float32)))
    out = np.empty_like(r)
    _lib.check(_lib.lib.wost_greens_norm(float(sigma_bar), _lib.fptr(r), r.shape[0], _lib.fptr(out)),
               "screenedGreensNorm2D")
    return out if np.ndim(R) else float(out[0])


__all__ = ["greensFunctionNorm2D", "screenedGreensNorm2D"]
