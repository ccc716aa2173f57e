"""DC-resistivity survey layer on top of the Walk-on-Stars solver.

The reference stops at electrode potentials (tests/testGeophysicalScenario.py
plots u at surface electrodes; the notebook, cells 3 and 21, differences
adjacent electrodes as a dipole-dipole line and imports SimPEG's
apparent_resistivity_from_voltage). This module turns potentials into survey
data:

* electrode arrays: dipole-dipole (receiver M_i = electrode i, N_i = i + 1,
  notebook cell 3) and Wenner quadripoles (A, M, N, B at spacing a);
* potential differences dV = u(M) - u(N) with Monte-Carlo standard errors;
* apparent resistivity rho_a = rho_bg * dV(model) / dV(homogeneous), the
  homogeneous solve using the background conductivity and the SAME random
  streams (common random numbers), SURVEY.md 8d;
* comparisons of two solutions of the same survey (e.g. GPU vs the CPU
  reference): RMSE of rho_a over resolved dipoles and the MC 1-sigma.
"""
from __future__ import annotations

import math
import os
import time
from dataclasses import dataclass

import numpy as np

from . import fields as F
from .scenarios import Scenario


def dipole_dipole_pairs(n_electrodes: int) -> np.ndarray:
    """[(m, n)] receiver dipoles of adjacent electrodes (notebook cell 3)."""
    i = np.arange(n_electrodes - 1)
    return np.stack([i, i + 1], axis=1)


def wenner_quadripoles(n_electrodes: int, a: int = 1) -> np.ndarray:
    """[(A, M, N, B)] Wenner-alpha quadripoles with electrode spacing a (in electrode steps)."""
    i = np.arange(n_electrodes - 3 * a)
    return np.stack([i, i + a, i + 2 * a, i + 3 * a], axis=1)


def dipole_dipole_quadripoles(n_electrodes: int, n_max: int = 4) -> np.ndarray:
    """[(A, B, M, N)] dipole-dipole quadripoles: current dipole (c, c+1), potential
    dipole (c+1+n, c+2+n) for separations n = 1..n_max (rows ordered by c, then n)."""
    rows = [(c, c + 1, c + 1 + n, c + 2 + n) for c in range(n_electrodes) for n in range(1, n_max + 1)
            if c + 2 + n < n_electrodes]
    return np.array(rows, dtype=np.int64).reshape(-1, 4)


def electrode_source(position, width: float, current: float = 1.0) -> F.Field:
    """Current injection at an electrode: a normalised Gaussian of standard deviation
    ``width`` (the reference's dcr_current_source form, tests/testGeophysicalScenario.py:11-33)."""
    norm = current / (2.0 * math.pi * width * width)
    return norm * F.gaussian((float(position[0]), float(position[1])), width)


def dipole_source(a, b, width: float, current: float = 1.0) -> F.Field:
    """+current at electrode position a, -current at b (notebook cell 17's dipole)."""
    return electrode_source(a, width, current) - electrode_source(b, width, current)


@dataclass
class DipoleData:
    dv: np.ndarray      # [P] potential differences u(M) - u(N)
    se: np.ndarray      # [P] their Monte-Carlo standard errors (walks of M and N are independent)


def potential_differences(u: np.ndarray, se: np.ndarray, pairs: np.ndarray) -> DipoleData:
    u = np.asarray(u, np.float64).ravel()
    se = np.asarray(se, np.float64).ravel()
    m, n = pairs[:, 0], pairs[:, 1]
    return DipoleData(u[m] - u[n], np.sqrt(se[m] ** 2 + se[n] ** 2))


@dataclass
class ApparentResistivity:
    rho_a: np.ndarray     # [P]
    se: np.ndarray        # [P] delta-method standard error (model and background treated as independent)
    resolved: np.ndarray  # [P] bool: both dV resolved (> 3 se) and rho_a's own error below a third of it


def apparent_resistivity(model: DipoleData, homogeneous: DipoleData, rho_bg: float) -> ApparentResistivity:
    """rho_a = rho_bg dV / dV_homogeneous. A dipole counts as resolved only when the
    ratio means something: the background's AND the model's potential difference
    exceed 3 standard errors, and rho_a's propagated error is below a third of it."""
    with np.errstate(divide="ignore", invalid="ignore"):
        ratio = model.dv / homogeneous.dv
        rel = np.sqrt((model.se / model.dv) ** 2 + (homogeneous.se / homogeneous.dv) ** 2)
        rho = rho_bg * ratio
        se = np.abs(rho) * rel
        ok = ((np.abs(homogeneous.dv) > 3.0 * homogeneous.se) & (np.abs(model.dv) > 3.0 * model.se)
              & np.isfinite(rho) & (se <= np.abs(rho) / 3.0))
    return ApparentResistivity(rho, se, ok)


def homogeneous(sc: Scenario, alpha_bg: float) -> Scenario:
    """The same survey with the conductivity field replaced by its background value.
    Solve it with the model solver's sigma_bar (``homogeneous_solver``): the delta-
    tracking collision test mu > sigma_bar G(r) and the sampler then match the
    model's, so walks with the same seed take identical paths and only their
    weights differ (common random numbers)."""
    return Scenario(sc.name + "_homogeneous", sc.dirichlet, sc.neumann, g=sc.g, f=sc.f, sigma=sc.sigma,
                    alpha=F.const(alpha_bg), points=sc.points, n_walks=sc.n_walks, max_steps=sc.max_steps,
                    eps=sc.eps, reference=sc.reference)


def homogeneous_solver(sc: Scenario, alpha_bg: float, model_solver, **kw):
    """WostSolver_2D of homogeneous(sc) with the model solver's sigma_bar (so that
    model and background walks of one seed share their paths)."""
    return homogeneous(sc, alpha_bg).solver(sigma_bar=model_solver.sigma_bar, **kw)


def paired_apparent_resistivity(model_walks: np.ndarray, bg_walks: np.ndarray, pairs: np.ndarray,
                                rho_bg: float) -> ApparentResistivity:
    """rho_a from per-walk values [E, W] of the model and the background solved on
    common random numbers (walk w of electrode e shares its path in both): the
    delta-method standard error then includes the model/background covariance of
    each electrode (electrodes are independent of each other)."""
    m = np.asarray(model_walks, np.float64)
    h = np.asarray(bg_walks, np.float64)
    W = m.shape[1]
    um, uh = m.mean(1), h.mean(1)
    vm, vh = m.var(1, ddof=1) / W, h.var(1, ddof=1) / W
    cmh = np.array([np.cov(m[e], h[e], ddof=1)[0, 1] for e in range(m.shape[0])]) / W
    i, j = pairs[:, 0], pairs[:, 1]
    A, B = um[i] - um[j], uh[i] - uh[j]
    vA, vB, cAB = vm[i] + vm[j], vh[i] + vh[j], cmh[i] + cmh[j]
    with np.errstate(divide="ignore", invalid="ignore"):
        R = A / B
        var = (vA - 2.0 * R * cAB + R * R * vB) / (B * B)
    rho = rho_bg * R
    se = rho_bg * np.sqrt(np.maximum(var, 0.0))
    # the ratio is resolved when B != 0 and its own delta-method error is below a third of it
    return ApparentResistivity(rho, se, (B != 0) & np.isfinite(rho) & (se <= np.abs(rho) / 3.0))


def replica_rho_a(model_walks: np.ndarray, bg_walks: np.ndarray, pairs: np.ndarray, rho_bg: float,
                  walks_per_replica: int) -> np.ndarray:
    """rho_a of independent replicas of walks_per_replica paired walks each: [R, P] with
    R = W // walks_per_replica (consecutive walks of every electrode form a replica)."""
    m = np.asarray(model_walks, np.float64)
    h = np.asarray(bg_walks, np.float64)
    R = m.shape[1] // walks_per_replica
    mm = m[:, :R * walks_per_replica].reshape(m.shape[0], R, walks_per_replica).mean(2)
    hm = h[:, :R * walks_per_replica].reshape(h.shape[0], R, walks_per_replica).mean(2)
    i, j = pairs[:, 0], pairs[:, 1]
    with np.errstate(divide="ignore", invalid="ignore"):
        return (rho_bg * (mm[i] - mm[j]) / (hm[i] - hm[j])).T


def matched_walk_pvalues(replicas: np.ndarray, observed: np.ndarray) -> np.ndarray:
    """Two-sided mid-p value of each observed rho_a among the replicas' values of the
    same dipole (non-finite replicas ignored): is the observation a plausible draw of
    the replicated estimator at the same walk count?"""
    out = np.full(len(observed), np.nan)
    for d in range(len(observed)):
        r = replicas[:, d]
        r = r[np.isfinite(r)]
        if len(r) == 0 or not np.isfinite(observed[d]):
            continue
        lt, eq = np.mean(r < observed[d]), np.mean(r == observed[d])
        out[d] = min(1.0, 2.0 * min(lt + 0.5 * eq, 1.0 - lt - 0.5 * eq))
    return out


@dataclass
class ReferenceSurvey:
    rho: ApparentResistivity     # the reference's rho_a per dipole-dipole receiver
    walks: int                   # walks per electrode the reference ran
    common_paths: bool           # model and background walks shared their paths
    u_model: np.ndarray          # [E] its electrode potentials
    u_background: np.ndarray


def reference_rho_a(path: str) -> ReferenceSurvey | None:
    """The reference's own dipole-dipole apparent resistivities of the C4 survey
    (tests/golden/rho_dcr_dipole.npz, made by tools/gen_fixtures.py --only rho: the
    reference's _solveUnified with its own torch/numpy RNG at all 48 electrodes, model
    conductivity and homogeneous alpha = 100), or None when the fixture is absent."""
    try:
        z = np.load(path, allow_pickle=False)
    except OSError:
        return None
    m, h = z["model_values"], z["background_values"]
    pairs = dipole_dipole_pairs(m.shape[0])
    rho = paired_apparent_resistivity(m, h, pairs, 1.0 / float(z["alpha_bg"]))
    return ReferenceSurvey(rho, int(z["n_walks"]), bool(z["common_paths"]), m.mean(1), h.mean(1))


@dataclass
class ReplaySurvey:
    """The reference's C4 survey replayed on libwost's Philox stream (tests/golden/
    rho_replay_dcr_dipole.npz, tools/gen_fixtures.py --only rho_replay): per-walk values
    and step counts [E, W] of the model and the alpha = 100 background, walk w of
    electrode e having global id e*W + w under ``seed``."""
    points: np.ndarray
    n_walks: int
    max_steps: int
    eps: float
    seed: int
    alpha_bg: float
    model_values: np.ndarray
    background_values: np.ndarray
    model_steps: np.ndarray
    background_steps: np.ndarray


def load_replay_survey(path: str) -> ReplaySurvey | None:
    try:
        z = np.load(path, allow_pickle=False)
    except OSError:
        return None
    return ReplaySurvey(z["points"], int(z["n_walks"]), int(z["max_steps"]), float(z["eps"]), int(z["seed"]),
                        float(z["alpha_bg"]), z["model_values"], z["background_values"], z["model_steps"],
                        z["background_steps"])


def compare_to_replay(vm: np.ndarray, vh: np.ndarray, sm: np.ndarray, sh: np.ndarray, ref: ReplaySurvey) -> dict:
    """Deterministic rho_a parity (no Monte-Carlo error): the device's per-walk values
    [E, W] and step counts on the replay's walks against the reference's, and the
    paired dipole-dipole rho_a of both (the same formula, the same walks)."""
    pairs = dipole_dipole_pairs(vm.shape[0])
    rb = 1.0 / ref.alpha_bg
    g = paired_apparent_resistivity(vm, vh, pairs, rb)
    r = paired_apparent_resistivity(ref.model_values, ref.background_values, pairs, rb)
    fin = np.isfinite(g.rho_a) & np.isfinite(r.rho_a)
    rel = np.abs(g.rho_a - r.rho_a) / np.maximum(np.abs(r.rho_a), 1e-300)
    wv = lambda a, b: np.abs(np.asarray(a, np.float64) - b) <= 1e-4 * np.abs(b) + 1e-6 * max(np.abs(b).max(), 1e-30)
    return {"fixture": "tests/golden/rho_replay_dcr_dipole.npz (reference _solveUnified on the Philox stream)",
            "electrodes": int(vm.shape[0]), "walks_per_electrode": int(vm.shape[1]),
            "dipoles": int(len(pairs)), "dipoles_compared": int(fin.sum()),
            "steps_identical": bool(np.array_equal(sm, ref.model_steps) and np.array_equal(sh, ref.background_steps)),
            "walk_values_within_1e-4": float(np.mean(np.concatenate([wv(vm, ref.model_values).ravel(),
                                                                      wv(vh, ref.background_values).ravel()]))),
            "rho_a_max_rel_diff": float(rel[fin].max()) if fin.any() else None,
            "rho_a_rmse": float(np.sqrt(np.mean((g.rho_a[fin] - r.rho_a[fin]) ** 2))) if fin.any() else None,
            "rho_a_reference": [float(x) for x in r.rho_a],
            "rho_a_gpu": [float(x) for x in g.rho_a]}


@dataclass
class WennerReplay:
    """The reference's C5 Wenner survey replayed on libwost's Philox stream (tests/golden/
    rho_replay_wenner_topography_physical.npz and, round 6, rho_replay_wenner_topography.npz:
    tools/gen_fixtures.py --only c5_rho_replay / c5_rho_replay_literal):
    setSourceTerm(transmitter q) + _solveUnified at both receivers (M, N) of each listed
    quadripole, the physical (or literal) conductivity and the alpha_bg background (the model's
    sigma_bar), each receiver's walks carrying the ids and the seed they have in
    run_wenner_survey(seed=survey_seed): walk w of electrode e has id (e - j0) W + w in
    its group's launch, seed group_seed(survey_seed, g). Values and steps [Q, 2, W]."""
    points: np.ndarray
    quadripoles: np.ndarray      # [Q, 4] (A, M, N, B)
    receivers: np.ndarray        # [Q, 2] electrodes M, N
    groups: np.ndarray           # [Q, 2] their electrode group
    n_walks: int
    max_steps: int
    eps: float
    survey_seed: int
    alpha_bg: float
    width: float
    sigma_bar: float
    model_values: np.ndarray
    background_values: np.ndarray
    model_steps: np.ndarray
    background_steps: np.ndarray
    source: str = "rho_replay_wenner_topography_physical.npz"   # the fixture file


def load_wenner_replay(path: str) -> WennerReplay | None:
    try:
        z = np.load(path, allow_pickle=False)
    except OSError:
        return None
    return WennerReplay(z["points"], z["quadripoles"], z["receivers"], z["groups"], int(z["n_walks"]),
                        int(z["max_steps"]), float(z["eps"]), int(z["survey_seed"]), float(z["alpha_bg"]),
                        float(z["width"]), float(z["sigma_bar"]), z["model_values"], z["background_values"],
                        z["model_steps"], z["background_steps"], os.path.basename(path))


def wenner_replay_subset(ref: WennerReplay, idx) -> WennerReplay:
    """The replay restricted to the quadripoles ``idx`` (a smaller CPU check)."""
    import dataclasses

    idx = np.asarray(idx)
    return dataclasses.replace(ref, quadripoles=ref.quadripoles[idx], receivers=ref.receivers[idx],
                               groups=ref.groups[idx], model_values=ref.model_values[idx],
                               background_values=ref.background_values[idx], model_steps=ref.model_steps[idx],
                               background_steps=ref.background_steps[idx])


def wenner_replay_walks(ref: WennerReplay, solve_walks, a: int = 1):
    """Per-walk values and steps [Q, 2, W] of the replay's receivers for the model (field
    0) and the background (field 1), from ``solve_walks(field, points, sources, W, seed,
    rows) -> (values [S, n, W], steps [n, W])`` run per electrode group exactly as
    run_wenner_survey launches it: the group's electrodes, its seed, the transmitters
    the listed quadripoles need there (one launch per group and field). ``rows`` are the
    group's electrodes (local indices) whose walks are read: a solver may skip the others."""
    E = len(ref.points)
    batches = list(wenner_batches(E, a))
    Q, W = len(ref.quadripoles), ref.n_walks
    out = [np.zeros((Q, 2, W)), np.zeros((Q, 2, W)), np.zeros((Q, 2, W), np.int64), np.zeros((Q, 2, W), np.int64)]
    for g in sorted(set(int(x) for x in ref.groups.ravel())):
        j0, j1, _, _ = batches[g]
        need = [(i, k) for i in range(Q) for k in range(2) if int(ref.groups[i, k]) == g]
        tx = sorted(set(int(ref.quadripoles[i, 0]) for i, _ in need))
        srcs = [dipole_source(ref.points[q], ref.points[q + 3 * a], ref.width) for q in tx]
        rows = sorted(set(int(ref.receivers[i, k]) - j0 for i, k in need))
        for f in (0, 1):
            v, st = solve_walks(f, ref.points[j0:j1], srcs, W, group_seed(ref.survey_seed, g), rows)
            for i, k in need:
                e = int(ref.receivers[i, k]) - j0
                out[f][i, k] = v[tx.index(int(ref.quadripoles[i, 0])), e]
                out[2 + f][i, k] = st[e]
    return tuple(out)


def solver_replay_walks(model_solver, background_solver, ref: WennerReplay):
    """wenner_replay_walks' solver on the device: the group's multi-source launch on the
    model or background handle (WostSolver_2D.solve_sources_walks), as the survey runs it."""
    def solve_walks(f, pts, srcs, W, seed, rows):
        s = (model_solver, background_solver)[f]
        return s.solve_sources_walks(pts, srcs, nWalks=W, maxSteps=ref.max_steps, eps=ref.eps, seed=seed)

    return solve_walks


def compare_wenner_replay(vm, vh, sm, sh, ref: WennerReplay, k_sigma: float = 4.0) -> dict:
    """rho_a parity of the C5 Wenner survey against the reference replayed on the same
    walks. C5's walks are chaotic: a last-ulp difference at a Neumann hit (the reference's
    torch cos/sin and 10k-element reductions round a few per cent of their results one ulp
    off the correctly rounded value) sends a walk elsewhere, so a few per cent of the walks
    leave the reference's path and end with an unrelated value. Each quadripole's rho_a
    difference comes from those walks alone, and is bounded by them: |drho| <= k_sigma *
    sigma_chaos + 1e-5 |rho|, sigma_chaos the delta-method error of rho_a over only the
    diverged walks (each a difference of two draws of the walk's distribution: 2 var per
    walk), plus what the identical walks may differ by (1e-3 of each value: the walk
    identity test's tolerance) and 1e-5 |rho|."""
    rb = 1.0 / ref.alpha_bg
    W = ref.n_walks
    rm, rh = np.asarray(ref.model_values, np.float64), np.asarray(ref.background_values, np.float64)
    vm, vh = np.asarray(vm, np.float64), np.asarray(vh, np.float64)
    scale_m, scale_h = max(np.abs(rm).max(), 1e-300), max(np.abs(rh).max(), 1e-300)
    same_m = (np.asarray(sm) == ref.model_steps) & (np.abs(vm - rm) <= 1e-3 * np.abs(rm) + 1e-5 * scale_m)
    same_h = (np.asarray(sh) == ref.background_steps) & (np.abs(vh - rh) <= 1e-3 * np.abs(rh) + 1e-5 * scale_h)
    div = ~(same_m & same_h)                                  # [Q, 2, W]

    def rho(m, h):
        A, B = m[:, 0].mean(1) - m[:, 1].mean(1), h[:, 0].mean(1) - h[:, 1].mean(1)
        with np.errstate(divide="ignore", invalid="ignore"):
            return rb * A / B, A, B

    g, Ag, _ = rho(vm, vh)
    r, A, B = rho(rm, rh)
    nd = div.sum(2)                                           # [Q, 2] diverged walks per receiver
    var_m, var_h = rm.var(2, ddof=1), rh.var(2, ddof=1)       # [Q, 2] walk-value variance per receiver
    with np.errstate(divide="ignore", invalid="ignore"):
        R = r / rb
        sig_a = np.sqrt((2.0 * nd * var_m).sum(1) / (W * W))   # dV(model) over the diverged walks
        sig = rb / np.abs(B) * np.sqrt(((2.0 * nd * var_m).sum(1) + R * R * (2.0 * nd * var_h).sum(1)) / (W * W))
        rel = np.abs(g - r) / np.abs(r)
        rel_a = np.abs(Ag - A) / np.abs(A)
        # the walks that did not diverge agree within the per-walk tolerance above
        e_m = ((1e-3 * np.abs(rm) + 1e-5 * scale_m) * ~div).sum(2).sum(1) / W
        e_h = ((1e-3 * np.abs(rh) + 1e-5 * scale_h) * ~div).sum(2).sum(1) / W
        tol = k_sigma * np.nan_to_num(sig) + rb / np.abs(B) * (e_m + np.abs(R) * e_h) + 1e-5 * np.abs(r)
    ok = np.abs(g - r) <= tol
    ok_a = np.abs(Ag - A) <= k_sigma * sig_a + e_m + 1e-5 * np.abs(A)
    clean = nd.sum(1) == 0
    return {"fixture": f"tests/golden/{ref.source} (reference setSourceTerm + _solveUnified on the Philox stream)",
            "quadripoles": int(len(r)), "walks_per_receiver": int(W),
            "walks_identical": float(1.0 - div.mean()),
            "steps_identical": float(np.mean(np.concatenate([(np.asarray(sm) == ref.model_steps).ravel(),
                                                              (np.asarray(sh) == ref.background_steps).ravel()]))),
            "quadripoles_without_diverged_walks": int(clean.sum()),
            "rel_diff_max_without_diverged_walks": {"rho_a": float(np.max(rel[clean])), "dv_model": float(np.max(
                rel_a[clean]))} if clean.any() else None,
            "tolerance": f"|d| <= {k_sigma} sigma_chaos + the identical walks' 1e-3 tolerance + 1e-5 |value| "
                         "(sigma_chaos: the delta-method error of the value over the diverged walks only)",
            "all_within_tolerance": bool(ok.all() and ok_a.all()),
            "rho_a": {"within_tolerance": int(ok.sum()),
                      "max_d_over_sigma_chaos": float(np.max(np.where(sig > 0, np.abs(g - r) / np.where(sig > 0, sig, 1.0),
                                                                      0.0))),
                      "reference": [float(x) for x in r], "gpu": [float(x) for x in g],
                      "rel_diff": [float(x) for x in rel], "sigma_chaos": [float(x) for x in sig]},
            "dv_model": {"within_tolerance": int(ok_a.sum()),
                         "max_d_over_sigma_chaos": float(np.max(np.where(sig_a > 0, np.abs(Ag - A) /
                                                                         np.where(sig_a > 0, sig_a, 1.0), 0.0))),
                         "reference": [float(x) for x in A], "gpu": [float(x) for x in Ag],
                         "rel_diff": [float(x) for x in rel_a], "sigma_chaos": [float(x) for x in sig_a]},
            "diverged_walks": [int(x) for x in nd.sum(1)]}


def compare_to_reference(gpu: ApparentResistivity, ref: ReferenceSurvey, replicas: np.ndarray | None = None) -> dict:
    """The north-star check (BASELINE.json): RMSE of rho_a(GPU) - rho_a(reference) over
    the dipoles the reference resolves, against the reference's 1-sigma Monte-Carlo
    error there (RMS), plus z-scores (RMS z <= 1.2, max |z| < 4). Dipoles
    the reference does not resolve are 'unpinned'.

    Two 1-sigmas are reported. ref_self_reported_1sigma_rms is the reference's own delta-method
    error from its 400 walks; delta-tracking walks are heavy-tailed (the rare walks
    that cross the conductivity anomalies carry the signal), and 400 of them mostly
    miss those events, so that estimate understates the error. With ``replicas``
    ([R, P] rho_a of independent GPU estimates at the reference's walk count)
    gpu_replica_1sigma_rms is the spread of the GPU's own 400-walk estimates; z-scores
    then use it too (z_rms, z_max), while z_rms_self_reported keeps the reference's
    own error. That bound is about rho_bg itself at 400 walks, so this statistical
    leg can hardly fail: the deterministic rho_a parity is compare_to_replay (the
    reference replayed on the same walks)."""
    r = ref.rho
    ok = r.resolved & gpu.resolved & np.isfinite(gpu.rho_a) & np.isfinite(r.rho_a)
    out = {"reference_walks_per_electrode": ref.walks, "dipoles": int(len(r.rho_a)), "resolved": int(ok.sum()),
           "unpinned": int(len(r.rho_a) - ok.sum()), "reference_common_paths": ref.common_paths}
    if not ok.any():
        out.update({"rmse": None, "ref_self_reported_1sigma_rms": None, "rmse_over_1sigma": None, "z_rms": None,
                    "z_max": None})
        return out
    d = gpu.rho_a[ok] - r.rho_a[ok]
    s = np.sqrt(gpu.se[ok] ** 2 + r.se[ok] ** 2)
    z = d / np.where(s > 0, s, 1.0)
    rmse = float(np.sqrt(np.mean(d * d)))
    one_sigma = float(np.sqrt(np.mean(r.se[ok] ** 2)))
    # (the self-reported error of 400 heavy-tailed walks understates the MC error by
    # orders of magnitude: kept for the record, not the north-star bound)
    out.update({"rmse": rmse, "ref_self_reported_1sigma_rms": one_sigma,
                "rmse_over_ref_self_reported_1sigma": rmse / one_sigma if one_sigma else None,
                "z_rms_self_reported": float(np.sqrt(np.mean(z * z))),
                "resolved_dipoles": [int(i) for i in np.nonzero(ok)[0]]})
    if replicas is not None:
        sd = np.nanstd(np.where(np.isfinite(replicas), replicas, np.nan), axis=0, ddof=1)[ok]
        s2 = np.sqrt(gpu.se[ok] ** 2 + sd ** 2)
        z2 = d / np.where(s2 > 0, s2, 1.0)
        rep_sigma = float(np.sqrt(np.mean(sd ** 2)))
        # the bound is the spread of the GPU's OWN replicas (wide: ~ rho_bg at 400 walks),
        # so this leg has little power; the deterministic parity is compare_to_replay
        out.update({"gpu_replica_1sigma_rms": rep_sigma,
                    "rmse_over_gpu_replica_1sigma": rmse / rep_sigma if rep_sigma else None,
                    "rmse_le_gpu_replica_1sigma": bool(rmse <= rep_sigma), "z_rms": float(np.sqrt(np.mean(z2 * z2))),
                    "z_max": float(np.max(np.abs(z2)))})
    else:
        out.update({"rmse_over_1sigma": out["rmse_over_ref_self_reported_1sigma"],
                    "rmse_le_1sigma": bool(rmse <= one_sigma),
                    "z_rms": out["z_rms_self_reported"], "z_max": float(np.max(np.abs(z)))})
    return out


@dataclass
class SurveyResult:
    pairs: np.ndarray
    model: DipoleData
    background: DipoleData
    rho: ApparentResistivity
    u_model: np.ndarray
    u_background: np.ndarray
    walk_steps: int


def run_dipole_dipole(sc: Scenario, alpha_bg: float, n_walks: int, seed: int = 0, device: int | None = None,
                      solvers=None) -> SurveyResult:
    """Solve the survey on the GPU: electrode potentials of the model and of the
    homogeneous background (same walk streams), then dV and rho_a = (1/alpha_bg) dV/dV_bg."""
    if solvers is None:
        sm = sc.solver(device=device)
        solvers = (sm, homogeneous_solver(sc, alpha_bg, sm, device=device))
    sm, sh = solvers
    _, st_m = sm.solve(sc.points, nWalks=n_walks, maxSteps=sc.max_steps, eps=sc.eps, seed=seed, return_stats=True)
    _, st_h = sh.solve(sc.points, nWalks=n_walks, maxSteps=sc.max_steps, eps=sc.eps, seed=seed, return_stats=True)
    pairs = dipole_dipole_pairs(len(sc.points))
    dm = potential_differences(st_m.mean, st_m.stderr, pairs)
    dh = potential_differences(st_h.mean, st_h.stderr, pairs)
    return SurveyResult(pairs, dm, dh, apparent_resistivity(dm, dh, 1.0 / alpha_bg), st_m.mean, st_h.mean,
                        st_m.total_steps + st_h.total_steps)


def compare(a: ApparentResistivity, b: ApparentResistivity) -> dict:
    """RMSE of rho_a between two solutions over dipoles resolved in both, the RMS
    of b's Monte-Carlo 1-sigma over the same dipoles (the north-star bound), and
    the z-scores z_i = (a_i - b_i) / sqrt(se_a^2 + se_b^2) (RMS z <= 1.2,
    max |z| < 4 for independent solutions)."""
    ok = a.resolved & b.resolved & np.isfinite(a.rho_a) & np.isfinite(b.rho_a)
    if not ok.any():
        return {"rmse": None, "mc_1sigma": None, "resolved": 0, "z_rms": None, "z_max": None}
    d = a.rho_a[ok] - b.rho_a[ok]
    s = np.sqrt(a.se[ok] ** 2 + b.se[ok] ** 2)
    z = np.where(s > 0, d / np.where(s > 0, s, 1.0), 0.0)
    return {"rmse": float(np.sqrt(np.mean(d * d))), "mc_1sigma": float(np.sqrt(np.mean(b.se[ok] ** 2))),
            "resolved": int(ok.sum()), "z_rms": float(np.sqrt(np.mean(z * z))), "z_max": float(np.max(np.abs(z)))}


@dataclass
class MultiSurveyResult:
    quadripoles: np.ndarray   # [Q, 4] (A, B, M, N)
    model: DipoleData         # [Q]
    background: DipoleData    # [Q]
    rho: ApparentResistivity  # [Q]
    u_model: np.ndarray       # [T, E] potential at every electrode for each transmitter dipole
    u_background: np.ndarray  # [T, E]
    transmitters: np.ndarray  # [T, 2] (A, B) of each row of u_*
    walk_steps: int


def run_dipole_dipole_survey(sc: Scenario, alpha_bg: float, n_walks: int, n_max: int = 4, width: float = 0.5,
                             seed: int = 0, device: int | None = None, solvers=None) -> MultiSurveyResult:
    """A full dipole-dipole pseudosection: one transmitter dipole (c, c+1) per
    electrode pair, every electrode's potential for each, model and homogeneous
    background. All transmitters are scored by the same walks
    (WostSolver_2D.solve_sources: the walks do not depend on the source), so the
    survey costs two walk sets per electrode instead of two per transmitter."""
    E = len(sc.points)
    quad = dipole_dipole_quadripoles(E, n_max)
    tx = np.unique(quad[:, :2], axis=0) if len(quad) else np.zeros((0, 2), np.int64)
    srcs = [dipole_source(sc.points[a], sc.points[b], width) for a, b in tx]
    if solvers is None:
        sm = sc.solver(device=device)
        solvers = (sm, homogeneous_solver(sc, alpha_bg, sm, device=device))
    sm, sh = solvers
    out = []
    steps = 0
    for s in (sm, sh):
        if not srcs:
            out.append((np.zeros((0, E)), np.zeros((0, E))))
            continue
        _, st = s.solve_sources(sc.points, srcs, nWalks=n_walks, maxSteps=sc.max_steps, eps=sc.eps, seed=seed,
                                return_stats=True)
        out.append((st.mean, st.stderr))
        steps += st.total_steps
    row = {(int(a), int(b)): k for k, (a, b) in enumerate(tx)}
    t = np.array([row[(int(a), int(b))] for a, b, _, _ in quad], dtype=np.int64)

    def dd(mean, se):
        if not len(quad):
            return DipoleData(np.zeros(0), np.zeros(0))
        m, n = quad[:, 2], quad[:, 3]
        return DipoleData(mean[t, m] - mean[t, n], np.sqrt(se[t, m] ** 2 + se[t, n] ** 2))

    dm, dh = dd(*out[0]), dd(*out[1])
    return MultiSurveyResult(quad, dm, dh, apparent_resistivity(dm, dh, 1.0 / alpha_bg), out[0][0], out[1][0], tx,
                             steps)


@dataclass
class WennerSurveyResult:
    quadripoles: np.ndarray   # [Q, 4] (A, M, N, B)
    model: DipoleData         # [Q] dV = u_A,B(M) - u_A,B(N) (transmitter A+ / B-)
    background: DipoleData    # [Q]
    rho: ApparentResistivity  # [Q] rho_bg dV / dV_background
    walk_steps: int           # model + background (all ranks with a communicator)
    launches: int             # multi-source solves (per field)
    kernel_ms: float          # walk-kernel time, both fields (this rank)
    local_walk_steps: int = 0  # this rank's walk-steps (= walk_steps on one GPU)
    # with a communicator, this rank's wall-clock ms summed over the groups' protocols:
    # wait_ms (the collective thread waiting for the local solves' results), agree_ms (the
    # agreement all-reduce: waits for the slowest rank), gather_ms, merge_ms
    phase_ms: dict | None = None


def wenner_batches(n_electrodes: int, a: int = 1, max_sources: int = 16):
    """Electrode groups of a Wenner survey for multi-source batching: quadripole q =
    (A, M, N, B) = (q, q+a, q+2a, q+3a) needs electrode M and N under transmitter q
    only, so electrode j is a receiver of transmitters j-a and j-2a. A group of
    max_sources - a consecutive electrodes [j0, j1) needs the transmitters
    [j0-2a, j1-a) -- at most max_sources of them -- and every electrode is walked once
    per field: yields (j0, j1, t0, t1) with transmitters clipped to [0, Q)."""
    Q = max(n_electrodes - 3 * a, 0)
    g = max(max_sources - a, 1)
    for j0 in range(0, n_electrodes, g):
        j1 = min(j0 + g, n_electrodes)
        t0, t1 = max(j0 - 2 * a, 0), min(j1 - a, Q)
        if t1 > t0:
            yield j0, j1, t0, t1


def group_seed(seed: int, g: int) -> int:
    """Seed of Wenner group g: groups' walk ids stay independent."""
    return (int(seed) * 0x9E3779B1 + g) & (2**64 - 1)


def prepare_survey_kernels(sc, solvers, srcs, batches, key=None, max_workers: int = 16) -> int:
    """Compile every group's field-specialised kernels before a survey's solves look them
    up (WostSolver_2D.prepare_sources), from a pool of threads whose compiles overlap in
    libwost's compile helper processes: a fresh process's first C5 survey compiles 34
    kernels, which the survey's own handle threads (2 per handle pair) would otherwise
    compile a few at a time. Group g's kernel of field f is prepared on the handle that
    solves it. ``key`` (hashable): skip when these solvers already prepared it. Returns the
    number of kernels prepared (0 when skipped)."""
    from concurrent.futures import ThreadPoolExecutor

    if not all(hasattr(s, "prepare_sources") for s in solvers):   # (host stand-ins)
        return 0
    if key is not None and all(key in getattr(s, "_prepared_surveys", ()) for s in solvers):
        return 0
    k = max(1, len(solvers) // 2)
    jobs = [(solvers[2 * (g % k) + f], srcs[t0:t1], j1 - j0)
            for g, (j0, j1, t0, t1) in enumerate(batches) for f in (0, 1)]
    with ThreadPoolExecutor(max_workers=max(1, min(max_workers, len(jobs)))) as ex:
        for fut in [ex.submit(s.prepare_sources, src, n) for s, src, n in jobs]:
            fut.result()
    if key is not None:
        for s in solvers:
            if not hasattr(s, "_prepared_surveys"):
                s._prepared_surveys = set()
            s._prepared_surveys.add(key)
    return len(jobs)


def _run_fields_distributed(sc, solvers, srcs, batches, n_walks, seed, comm, record, concurrent=True,
                            phase_ms: dict | None = None):
    """The model and background fields of a multi-source survey across the ranks of one
    communicator. Worker threads (one per field and handle pair, or one per handle pair
    without ``concurrent``) solve this rank's walk range of every group
    (WostSolver_2D.solve_range with the group's sources installed) and hand the block
    rows over; THIS thread then runs
    libwost's protocol (distributed.run_protocol: agreement all-reduce, all-gather,
    ordered merge) for group 0 model, group 0 background, group 1 model, ... -- the same
    collective sequence on every rank, whatever the threads' timing. A local failure
    travels through the protocol's agreement (every rank raises; no rank waits)."""
    import queue
    import threading

    from . import _lib
    from .comm import shard_walk_range
    from .distributed import run_protocol, solve_key
    from .solvers.WoStSolver import SolveStats, _stats_of_multi

    R, rank = int(comm.n_ranks), int(comm.rank)
    w0, w1 = shard_walk_range(int(n_walks), R, rank)
    G = len(batches)
    slots = [[queue.Queue(maxsize=1) for _ in range(G)] for _ in range(2)]
    stop = threading.Event()

    def local(tasks, k):
        for f, g in tasks:
            j0, j1, t0, t1 = batches[g]
            if stop.is_set():
                slots[f][g].put((None, RuntimeError("survey stopped"), None))
                continue
            s = solvers[2 * (g % k) + f]
            try:
                if len(srcs[t0:t1]) > _lib.WOST_MAX_SOURCES:
                    raise ValueError(f"group {g} needs {t1 - t0} sources (> {_lib.WOST_MAX_SOURCES})")
                blocks, tm = None, {"total_steps": 0, "walk_kernel_ms": 0.0, "total_ms": 0.0}
                if w1 > w0:
                    with s.sources_installed(s.source_fields(srcs[t0:t1])):
                        blocks = s.solve_range(sc.points[j0:j1], int(n_walks), w0, w1, sc.max_steps, sc.eps,
                                               group_seed(seed, g))
                        tm = s.last_timing
                slots[f][g].put((blocks, None, tm))
            except Exception as e:   # noqa: BLE001 -- reported through the protocol
                slots[f][g].put((None, e, None))

    k = max(1, len(solvers) // 2)   # handles per field: worker (f, w) solves the groups g = w mod k
    work = [[(f, g) for g in range(G) if g % k == w for f in (0, 1)] for w in range(k)]
    if concurrent:
        work = [[(f, g) for (f, g) in wl if f == ff] for wl in work for ff in (0, 1)]
    threads = [threading.Thread(target=local, args=(wl, k), daemon=True) for wl in work]
    for t in threads:
        t.start()
    try:
        for g, (j0, j1, t0, t1) in enumerate(batches):
            S = t1 - t0
            for f in (0, 1):
                t_wait = time.perf_counter()
                blocks, err, tm = slots[f][g].get()
                if phase_ms is not None:
                    phase_ms["wait_ms"] = phase_ms.get("wait_ms", 0.0) + 1e3 * (time.perf_counter() - t_wait)

                def solve_range(a, b, blocks=blocks, err=err):
                    if err is not None:
                        raise err
                    if (a, b) != (w0, w1):
                        raise ValueError(f"protocol asked for walks [{a}, {b}), this rank solved [{w0}, {w1})")
                    return blocks

                key = solve_key(group_seed(seed, g), sc.eps, sc.max_steps, sc.points[j0:j1])
                ph = {}
                sums, _, all_steps = run_protocol(R, rank, j1 - j0, int(n_walks), 2 * S + 1, solve_range,
                                                  comm.allreduce, comm.allgather, key=key, phases=ph)
                if phase_ms is not None:
                    for name in ("agree_ms", "gather_ms", "merge_ms"):
                        phase_ms[name] = phase_ms.get(name, 0.0) + ph[name]
                stats = _stats_of_multi(sums, int(n_walks))
                st = SolveStats(mean=np.stack([x.mean for x in stats]), stderr=np.stack([x.stderr for x in stats]),
                                mean_steps=stats[0].mean_steps, walks=int(n_walks), total_steps=int(all_steps),
                                kernel_ms=float(tm["walk_kernel_ms"]) if tm else 0.0,
                                total_ms=float(tm["total_ms"]) if tm else 0.0)
                record(f, g, st, int(tm["total_steps"]) if tm else 0)
    finally:
        stop.set()
        for t in threads:   # the workers only solve locally: they always finish
            t.join()


def run_wenner_survey(sc: Scenario, alpha_bg: float, n_walks: int, a: int = 1, width: float = 0.5, seed: int = 0,
                      device: int | None = None, solvers=None, concurrent: bool = True,
                      comm=None) -> WennerSurveyResult:
    """A Wenner-alpha line over the scenario's electrodes: transmitter
    q injects +1 A at electrode q and -1 A at q+3a (dipole_source, Gaussians of std
    `width`), receivers M = q+a, N = q+2a. Multi-source batching (wenner_batches): each
    electrode is walked once per field and its walks score the (<= 16) transmitters it
    receives, model and homogeneous background on common random numbers (the same seed
    per group). Group g uses seed (seed, g) so that groups' walk ids stay independent.
    With ``concurrent`` the model and background fields run in two host threads, each on
    its own solver handle and HIP stream (libwost's calls release the GIL), so that two
    launches share the GPU: a group's launch (<= 16 electrodes) under-fills it at small
    walk counts, and its last walks run while the other launch fills the CUs.
    ``solvers`` may hold several (model, background) handle pairs; group g then runs on
    pair g mod k, one thread per handle, so that 2k launches share the GPU. The results
    do not depend on either.

    ``comm`` (collective; every rank calls with the same arguments): a
    dcrmontecarlo_amd.comm.Communicator (or any object with its ``n_ranks``, ``rank``,
    ``allreduce`` and ``allgather``). Every group is solved across the ranks by walk
    ranges, the results bitwise the one-GPU survey's (_run_fields_distributed): the two
    fields' local walk-range solves run concurrently in two threads, while ONE thread
    issues every collective, in a fixed order -- group by group, model before
    background -- so that no two ranks can interleave them differently."""
    E = len(sc.points)
    quad = wenner_quadripoles(E, a)
    Q = len(quad)
    srcs = [dipole_source(sc.points[q], sc.points[q + 3 * a], width) for q in range(Q)]
    if solvers is None:
        sm = sc.solver(device=device)
        solvers = (sm, homogeneous_solver(sc, alpha_bg, sm, device=device))
    if isinstance(comm, (tuple, list)):
        raise ValueError("run_wenner_survey takes one communicator: the fields' collectives are issued in a fixed "
                         "order on it (a pair of communicators driven from two threads can deadlock)")
    mean = [np.full((Q, E), np.nan), np.full((Q, E), np.nan)]
    se = [np.full((Q, E), np.nan), np.full((Q, E), np.nan)]
    batches = list(wenner_batches(E, a))
    acc = [[0, 0.0, 0], [0, 0.0, 0]]   # per field: walk-steps (all ranks), walk-kernel ms, walk-steps (this rank)

    import threading

    lock = threading.Lock()
    if len(solvers) < 2 or len(solvers) % 2:
        raise ValueError("solvers: (model, background) handle pairs, e.g. (model, background) or "
                         "(model, background, model2, background2)")
    k = len(solvers) // 2   # handle pairs: group g runs on pair g mod k
    # the groups' kernels, compiled at once on a cold start (a no-op for prepared solvers)
    prepare_survey_kernels(sc, solvers, srcs, batches,
                           key=("wenner", a, float(width), hash(np.ascontiguousarray(sc.points).tobytes())))

    def record(f, g, st, local):
        j0, j1, t0, t1 = batches[g]
        with lock:
            mean[f][t0:t1, j0:j1] = st.mean
            se[f][t0:t1, j0:j1] = st.stderr
            acc[f][0] += st.total_steps
            acc[f][1] += st.kernel_ms
            acc[f][2] += local

    def field(f, w):
        s = solvers[2 * w + f]
        for g, (j0, j1, t0, t1) in enumerate(batches):
            if g % k != w:
                continue
            _, st = s.solve_sources(sc.points[j0:j1], srcs[t0:t1], nWalks=n_walks, maxSteps=sc.max_steps,
                                    eps=sc.eps, seed=group_seed(seed, g), return_stats=True)
            record(f, g, st, st.total_steps)

    phase_ms = None
    if comm is not None:
        phase_ms = {"wait_ms": 0.0, "agree_ms": 0.0, "gather_ms": 0.0, "merge_ms": 0.0}
        _run_fields_distributed(sc, solvers, srcs, batches, n_walks, seed, comm, record, concurrent, phase_ms)
    elif concurrent:
        from concurrent.futures import ThreadPoolExecutor

        with ThreadPoolExecutor(max_workers=2 * k) as ex:
            for fut in [ex.submit(field, f, w) for w in range(k) for f in range(2)]:
                fut.result()
    else:
        for w in range(k):
            for f in range(2):
                field(f, w)
    steps, kms, launches = acc[0][0] + acc[1][0], acc[0][1] + acc[1][1], len(batches)
    q = np.arange(Q)
    M, N = quad[:, 1], quad[:, 2]
    dm = DipoleData(mean[0][q, M] - mean[0][q, N], np.sqrt(se[0][q, M] ** 2 + se[0][q, N] ** 2))
    dh = DipoleData(mean[1][q, M] - mean[1][q, N], np.sqrt(se[1][q, M] ** 2 + se[1][q, N] ** 2))
    return WennerSurveyResult(quad, dm, dh, apparent_resistivity(dm, dh, 1.0 / alpha_bg), steps, launches, kms,
                              acc[0][2] + acc[1][2], phase_ms)
