"""Import-path shim: the reference's ``geometry`` package (reference geometry/__init__.py).
Re-exports the MI355X polyline classes (dcrmontecarlo_amd.geometry)."""
from dcrmontecarlo_amd.geometry import PolyLines, PolyLinesSimple

__all__ = ["PolyLines", "PolyLinesSimple"]
