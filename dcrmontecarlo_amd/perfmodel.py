"""Algorithmic work model of one walk-step (for roofline reporting).

A walk-step is one iteration of the reference's while loop
(solvers/WoStSolver.py:206-291). Its floating-point work is counted from the
operations that loop performs -- not from the instructions the compiler emits
-- with the SURVEY.md 8d convention: add/sub/mul = 1, FMA = 2,
div/sqrt/exp/log/sin/cos/atan2 = 1 each, comparisons and the Philox integer
work = 0. Per component (derivations in DESIGN.md, "Roofline"):

  closest point on a segment (PolylinesSimple.py:37-47)        23 per Dirichlet segment, +1 sqrt
  silhouette test of an interior vertex (:63-81)               15 per Neumann interior vertex
  ray-segment test (:117-130)                                  15 per Neumann segment, +14 setup/exit
  direction theta, cos, sin (WoStSolver.py:226-232)             4
  next point without Neumann (:238)                             4
  source sample, clip test (:244-250)                          22
  Poisson contribution f r^2/4 (:256-258)                       4 + f
  delta: Green's norm via i0e Chebyshev (utils.py:43-44)       74
  delta: contribution (:253-258)                                6 + f + jet(alpha)
  delta: collision update incl. sigma' (:271-284)              28 + sigma
Field costs: per term 3, per factor value / jet as in _FACTOR_VALUE / _FACTOR_JET.
"""
from __future__ import annotations

# per-factor costs (value, jet incl. the product-rule multiply)
_FACTOR_VALUE = {1: None, 2: 16, 3: 5, 4: 5, 5: 8, 6: 12, 7: 4, 8: 5, 9: 58}
_FACTOR_JET = {1: None, 2: 50, 3: 32, 4: 32, 5: 36, 6: 50, 7: 24, 8: 25, 9: 160}
# 9 (tabulated): per axis 16 for the Catmull-Rom weights (+18 derivatives, +12
# second derivatives for the jet); 4 rows x 4 taps multiply-add = 32 (x3 for the
# jet) plus the 4-row combination

FP32_PEAK_TFLOPS = 157.3      # MI355X vector (= dense MFMA) FP32, MI355X_MICROARCH.md
HBM_PEAK_GBS = 8000.0         # MI355X HBM3E spec


def _field_cost(field, jet: bool) -> float:
    if field is None:
        return 0.0
    total = 0.0
    for coef, first, n in field.pack()[0]:
        total += 3.0 if not jet else 6.0
    for kind, p in field.pack()[1]:
        if kind == 1:
            e = int(p[0]) + int(p[1])
            total += (e + 1) if not jet else (3 * e + 28)
        else:
            total += (_FACTOR_VALUE if not jet else _FACTOR_JET)[kind]
    return total


TREE_MIN_SEGMENTS = 64       # include/wost.h WOST_TREE_MIN_SEGMENTS_DEFAULT


def flops_per_step(scenario):
    """Model FLOPs of one walk-step of the scenario's kernel variant, or None when
    the Neumann queries go through the segment tree: its work depends on the
    traversal, and the reference's full-scan count would exceed the peak."""
    if scenario.neumann is not None and scenario.neumann.shape[0] - 1 >= TREE_MIN_SEGMENTS:
        return None
    nd = scenario.dirichlet.shape[0]
    F = 23.0 * (nd - 1) + 1.0
    neu = scenario.neumann is not None
    if neu:
        nn = scenario.neumann.shape[0]
        F += 15.0 * max(nn - 2, 0) + 1.0
        F += 15.0 * (nn - 1) + 14.0
    else:
        F += 4.0
    F += 4.0
    delta = scenario.sigma is not None or scenario.alpha is not None
    if scenario.f is not None:
        F += 22.0 + _field_cost(scenario.f, jet=False)
        if delta:
            F += 74.0 + 6.0 + _field_cost(scenario.alpha, jet=True)
            F += 28.0 + _field_cost(scenario.sigma, jet=False)
        else:
            F += 4.0
    return F


def hbm_bytes_per_walk() -> float:
    """Algorithmic HBM traffic of the walk kernel per walk: the per-walk result
    (float value + uint32 step count) it writes. Geometry, sampler table, field
    program and query points are read once per workgroup into LDS / the scalar
    cache. (rocprofv3 on C4: WRITE_SIZE 413 MB per 48M-walk launch, FETCH_SIZE
    0.4 MB after the gfx950 x2 correction -- profiles/r01_jit/.)"""
    return 8.0
