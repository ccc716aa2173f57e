"""Walk-on-Stars solver (reference: solvers/__init__.py, WoStSolver.py)."""
from .WoStSolver import SolveStats, WostSolver_2D

__all__ = ["WostSolver_2D", "SolveStats"]
