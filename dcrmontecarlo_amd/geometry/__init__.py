"""Polyline boundaries (reference: geometry/__init__.py, Polylines.py, PolylinesSimple.py)."""
from .Polylines import PolyLines
from .PolylinesSimple import PolyLinesSimple

__all__ = ["PolyLines", "PolyLinesSimple"]
