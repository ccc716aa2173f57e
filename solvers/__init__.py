"""Import-path shim: the reference's ``solvers`` package (reference solvers/__init__.py).

A reference scenario script that does ``from solvers.WoStSolver import
WostSolver_2D`` with this repository's root on sys.path gets the MI355X solver
(dcrmontecarlo_amd) without editing its imports. Nothing is implemented here.
"""
from dcrmontecarlo_amd.solvers import SolveStats, WostSolver_2D

__all__ = ["WostSolver_2D", "SolveStats"]
