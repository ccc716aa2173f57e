"""Import-path shim for ``geometry.PolylinesSimple`` (reference geometry/PolylinesSimple.py:199-307):
the GPU-backed PolyLinesSimple of dcrmontecarlo_amd.geometry."""
from dcrmontecarlo_amd.geometry.PolylinesSimple import PolyLinesSimple

__all__ = ["PolyLinesSimple"]
