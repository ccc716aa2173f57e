"""Import-path shim for ``solvers.WoStSolver`` (reference solvers/WoStSolver.py:15-353):
re-exports the MI355X ``WostSolver_2D`` (dcrmontecarlo_amd.solvers.WoStSolver)."""
from dcrmontecarlo_amd.solvers.WoStSolver import SolveStats, WostSolver_2D, kernel_source, stats_from_sums

__all__ = ["WostSolver_2D", "SolveStats", "kernel_source", "stats_from_sums"]
