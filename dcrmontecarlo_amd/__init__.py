"""dcrmontecarlo_amd -- MI355X-native Walk-on-Stars solver for 2-D DC resistivity.

Drop-in for the hot path of Tsuchijo/DCRMonteCarlo: ``WostSolver_2D`` and
``PolyLinesSimple`` keep the reference's API while the per-walk loop runs in
hand-written gfx950 HIP kernels (libwost.so, C ABI in include/wost.h).
"""
from . import fields
from .geometry import PolyLines, PolyLinesSimple
from .solvers import SolveStats, WostSolver_2D

__all__ = ["WostSolver_2D", "SolveStats", "PolyLines", "PolyLinesSimple", "fields"]
__version__ = "0.1.0"
