"""Import-path shim for ``geometry.Polylines`` (reference geometry/Polylines.py:8-63)."""
from dcrmontecarlo_amd.geometry.Polylines import PolyLines

__all__ = ["PolyLines"]
