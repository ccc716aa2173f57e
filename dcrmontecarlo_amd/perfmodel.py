"""Algorithmic work model of one walk-step (for roofline reporting).

A walk-step is one iteration of the reference's while loop
(solvers/WoStSolver.py:206-291). The roofline fraction in bench.py uses
SURVEY.md 8(d)'s FLOP model v1 verbatim (convention: add/mul = 1, FMA = 2,
sqrt/rcp/exp/log/sin/cos = 1, compares and Philox integer work = 0):

  F_geom = 12 S_D + 15 (V_N - 2)^+ + 14 S_N
           (closest point per Dirichlet segment, silhouette test per interior
            Neumann vertex, ray test per Neumann segment)
  F_mode = Laplace ~10 | Poisson ~25 + f | delta ~150 (i0e ~120 included) + fields

with the per-config totals SURVEY 8(d) quotes:

  C1a Laplace ~58, C2 Poisson ~75, C3 variable coefficients ~1,150,
  C4 DCR ~350, C5 brute force ~290,000

The kernel no longer evaluates the i0e series (the Green's norm is an LDS
table lookup), so for delta tracking the model counts ~120 FLOP
the kernel does not execute; the fraction is reported against SURVEY's model
anyway, so that it is reproducible from SURVEY 8(d) and nothing else.

For configurations SURVEY does not quote, ``flops_per_step`` evaluates the same
v1 formula with the fields costed per term / factor (``_field_cost``).
"""
from __future__ import annotations

# SURVEY.md 8(d) "Per config (FLOP/step)"
SURVEY_FLOPS = {
    "laplace_square": 58.0,
    "poisson_square": 75.0,
    "variable_coefficients": 1150.0,
    "dcr_dipole": 350.0,
    "dcr_dipole_homogeneous": 350.0,
    "wenner_topography": 290000.0,
}

# per-factor costs (value, jet incl. the product-rule multiply), for fields of
# configurations SURVEY 8(d) does not quote
_FACTOR_VALUE = {1: None, 2: 16, 3: 5, 4: 5, 5: 8, 6: 12, 7: 4, 8: 5, 9: 58}
_FACTOR_JET = {1: None, 2: 50, 3: 32, 4: 32, 5: 36, 6: 50, 7: 24, 8: 25, 9: 160}

FP32_PEAK_TFLOPS = 157.3      # MI355X vector (= dense MFMA) FP32, MI355X_MICROARCH.md
HBM_PEAK_GBS = 8000.0         # MI355X HBM3E spec
# issue model (MI355X_MICROARCH.md, 'vector-instruction ISSUE cost'): a wave64
# VALU instruction occupies its SIMD for 2 cycles, a transcendental
# (v_exp/log/rcp/rsq/sqrt/sin/cos) for 8
CLOCK_GHZ = 2.4
N_SIMDS = 256 * 4
VALU_ISSUE_CYC = 2.0
TRANS_ISSUE_CYC = 8.0


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


def flops_per_step(scenario) -> float:
    """SURVEY 8(d) v1 FLOPs of one walk-step: the quoted per-config total when
    SURVEY quotes one for this scenario, else the v1 formula."""
    if scenario.name in SURVEY_FLOPS:
        return SURVEY_FLOPS[scenario.name]
    sd = scenario.dirichlet.shape[0] - 1
    F = 12.0 * sd
    if scenario.neumann is not None:
        vn = scenario.neumann.shape[0]
        F += 15.0 * max(vn - 2, 0) + 14.0 * (vn - 1)
    delta = scenario.sigma is not None or scenario.alpha is not None
    if delta:
        F += 150.0 + _field_cost(scenario.f, False) + _field_cost(scenario.alpha, True) \
            + _field_cost(scenario.sigma, False)
    elif scenario.f is not None:
        F += 25.0 + _field_cost(scenario.f, False)
    else:
        F += 10.0
    return F


I0E_FLOPS = 120.0   # the i0e series SURVEY 8(d) counts in the delta-tracking overhead


def executed_flops_per_step(scenario) -> float:
    """The v1 model without the ~120 FLOP i0e series that delta tracking's step no
    longer evaluates (the screened Green's norm is an LDS table lookup):
    the FP32 work the kernel actually executes per step, by the same convention."""
    f = flops_per_step(scenario)
    delta = scenario.sigma is not None or scenario.alpha is not None
    return f - I0E_FLOPS if delta else f


# v_mad_u64_u32 (Philox's 32x32 -> 64-bit products) issues in ~7.1 SIMD cycles, not 2:
# 9.66 cycles with its xor against 2.56 for v_fma_f32 (profiles/r02_fields/isa_rates.log,
# tools/microbench/isa_rates.hip). A walk-step draws one Philox4x32-10 block: 18 of them
# (rounds 0-1 hoisted per walk, tests/test_philox_split.py), counted statically.
MAD64_ISSUE_CYC = 7.1
PHILOX_MAD64_PER_STEP = 18


def issue_fraction(valu_per_wave_step: float, trans_per_wave_step: float, steps_per_s: float,
                   mad64_per_wave_step: float = 0.0) -> dict:
    """VALU issue-rate roofline: the SIMD cycles one wave-step's instructions occupy,
    (VALU - TRANS) x 2 + TRANS x 8, times the wave-steps per second, over the chip's
    SIMD cycles per second. With mad64_per_wave_step, also the same line with those
    v_mad_u64_u32 at their measured cost (frac_mad64_measured)."""
    cyc = (valu_per_wave_step - trans_per_wave_step) * VALU_ISSUE_CYC + trans_per_wave_step * TRANS_ISSUE_CYC
    avail = N_SIMDS * CLOCK_GHZ * 1e9
    used = cyc * steps_per_s / 64.0
    out = {"bound": "valu-issue", "cycles_per_wave_step": cyc, "achieved_simd_cycles_per_s": used,
           "peak_simd_cycles_per_s": avail, "frac": used / avail,
           "ceiling_walk_steps_per_s": avail * 64.0 / cyc if cyc > 0 else None}
    if mad64_per_wave_step:
        cyc2 = cyc + mad64_per_wave_step * (MAD64_ISSUE_CYC - VALU_ISSUE_CYC)
        out.update({"mad64_per_wave_step": mad64_per_wave_step, "mad64_issue_cycles": MAD64_ISSUE_CYC,
                    "cycles_per_wave_step_mad64_measured": cyc2,
                    "frac_mad64_measured": cyc2 * steps_per_s / 64.0 / avail})
    return out


def hbm_bytes_per_walk() -> float:
    """Algorithmic HBM traffic of the walk kernel per walk: the per-walk result
    (float value + uint32 step count) it writes. Geometry, sampler table, field
    program and query points are read once per workgroup into LDS / the scalar
    cache."""
    return 8.0
