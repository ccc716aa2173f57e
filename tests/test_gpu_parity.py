"""Parity of libwost's gfx950 kernels with the reference (golden vectors produced
by running the reference itself) and with the CPU oracle. All calls go through
the C ABI (ctypes); there is no fallback path.

Tolerances (float32 walk arithmetic like the reference's tensors):
  * geometry: distances/points within 8 ulps of the largest coordinate, ray
    "times" rtol 1e-5, silhouette masks >= 99.9% identical;
  * replay (the reference run on the same Philox stream): identical step counts
    for every walk, >= 99% of per-walk values within 1e-4, all within 2e-3;
  * device vs oracle: per-scenario floor of identical walks (99%, 97% for the
    chaotic variable-coefficient scenario) and per-point means within 0.5 MC
    standard errors;
  * statistics vs the reference's own RNG: bootstrap p > 1e-3 for every point
    (means and walk lengths) -- the north star's "within the MC standard error".
"""
import numpy as np
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu

SCEN = ["laplace_square", "manufactured_polynomial", "poisson_square", "variable_coefficients", "dcr_dipole",
        "notebook_dcr"]


def _solver_for(name, z=None, **kw):
    from dcrmontecarlo_amd import scenarios as S
    from dcrmontecarlo_amd.geometry import PolyLinesSimple
    from dcrmontecarlo_amd.solvers import WostSolver_2D

    sc = S.ALL[name]()
    D = z["dirichlet"] if z is not None and "dirichlet" in z else sc.dirichlet
    N = (z["neumann"] if "neumann" in z else None) if z is not None else sc.neumann
    return sc, WostSolver_2D(PolyLinesSimple(D), sc.g, PolyLinesSimple(N) if N is not None else None,
                             source=sc.f, sigma=sc.sigma, alpha=sc.alpha, **kw)


# ---------------------------------------------------------------- geometry
GEOMS = ["unit_square", "square2", "square15", "circle33", "box100", "top_segment", "open_u", "zigzag", "kat_tri",
         "topo10k"]


@pytest.mark.parametrize("geom", GEOMS)
def test_geometry_kats_device(gpu_available, geom):
    from dcrmontecarlo_amd.geometry import PolyLinesSimple

    z = golden("geometry_kats.npz")
    V, P, Dd, R = (z[f"{geom}__{k}"] for k in ("verts", "points", "dirs", "radii"))
    poly = PolyLinesSimple(V)
    tol = 8 * np.finfo(np.float32).eps * max(1.0, float(np.abs(V).max()))   # a few ulps of the coordinates
    d = poly.distance(P)
    np.testing.assert_allclose(d, z[f"{geom}__distance"], rtol=2e-6, atol=tol)
    sd = poly.silhouetteDistance(P)
    ref_sd = z[f"{geom}__silhouette_distance"]
    assert np.array_equal(np.isinf(sd), np.isinf(ref_sd)) or np.mean(np.isinf(sd) == np.isinf(ref_sd)) > 0.98
    fin = np.isfinite(sd) & np.isfinite(ref_sd)
    np.testing.assert_allclose(sd[fin], ref_sd[fin], rtol=2e-6, atol=tol)
    if V.shape[0] > 2:
        m = poly.isSilhouette(P)
        assert np.mean(m == z[f"{geom}__is_silhouette"].astype(bool)) > 0.999
    t = poly.rayIntersection(P, Dd)
    rt = z[f"{geom}__ray_intersection"]
    assert np.mean(np.isinf(t) == np.isinf(rt)) > 0.999
    both = np.isfinite(t) & np.isfinite(rt)
    np.testing.assert_allclose(t[both], rt[both], rtol=1e-5, atol=1e-6)
    hp, nrm, found = poly.intersectPolylines(P, Dd, R)
    ri = z[f"{geom}__intersect"]
    agree = found == (ri[:, 4] != 0)
    assert agree.mean() > 0.99
    np.testing.assert_allclose(hp[agree], ri[agree, 0:2], rtol=1e-5, atol=tol)
    np.testing.assert_allclose(nrm[agree], ri[agree, 2:4], atol=1e-6)


def test_reference_inline_kats_device(gpu_available):
    """The reference's own inline tests (geometry/PolylinesSimple.py:309-357)."""
    from dcrmontecarlo_amd.geometry import PolyLinesSimple

    sq = PolyLinesSimple(np.array([[0, 0], [1, 0], [1, 1], [0, 1], [0, 0]], np.float32))
    assert abs(sq.distance(np.array([0.5, 0.5], np.float32)) - 0.5) < 1e-6
    tri = PolyLinesSimple(np.array([[0, 0], [1, 1], [2, 0]], np.float32))
    assert list(tri.isSilhouette(np.array([1.5, 0.6], np.float32))) == [True]
    assert abs(tri.silhouetteDistance(np.array([1.5, 0.6], np.float32)) - np.hypot(0.5, 0.4)) < 1e-6
    t = sq.rayIntersection(np.array([0.5, 0.5], np.float32), np.array([1.0, 0.0], np.float32))
    np.testing.assert_allclose(t, [np.inf, 0.5, np.inf, np.inf], atol=1e-6)
    p, n, found = sq.intersectPolylines(np.array([0.5, 0.5], np.float32), np.array([1.0, 0.0], np.float32), 2.0)
    np.testing.assert_allclose(p, [1.0, 0.5], atol=1e-6)
    np.testing.assert_allclose(n, [-1.0, 0.0], atol=1e-6)
    assert found


# ---------------------------------------------------------------- fields, sigma', sigma_bar
@pytest.mark.parametrize("name", SCEN)
def test_fields_device(gpu_available, name):
    z = golden(f"fields_{name}.npz")
    sc, s = _solver_for(name, z)
    P = z["points"]
    for key, slot in (("g", "g"), ("f", "f"), ("alpha", "alpha"), ("sigma", "sigma")):
        if key not in z.files:
            continue
        if slot in ("alpha", "sigma") and not s.use_delta_tracking:
            continue
        ref = z[key]
        got = s.eval_field(slot, P)[:, 0].astype(np.float64)
        scale = max(np.abs(ref).max(), 1e-30)
        np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-6 * scale, err_msg=f"{name}.{key}")
    if "sigma_bar" in z.files:
        assert s.sigma_bar == pytest.approx(float(z["sigma_bar"]), rel=1e-5)
        sp = s.eval_field("sigma_prime", P)[:, 0].astype(np.float64)
        ref = z["sigma_prime"]
        fin = np.isfinite(ref)
        scale = np.abs(ref[fin]).max()
        np.testing.assert_allclose(sp[fin], ref[fin], rtol=2e-3, atol=1e-5 * scale, err_msg=f"{name}.sigma'")


# ---------------------------------------------------------------- sampler
def test_sampler_table_vs_oracle(gpu_available):
    from oracle import oracle as O

    for name, sb in (("poisson_square", None), ("variable_coefficients", 3.217497020959854), ("dcr_dipole", 10.0)):
        sc, s = _solver_for(name)
        tab = s.sampler_table()
        ref = O.sampler_nodes(sb is not None, sb or 0.0)
        np.testing.assert_allclose(tab, ref, rtol=0, atol=2e-6, err_msg=name)
        assert np.all(np.diff(tab) >= 0)


# ---------------------------------------------------------------- replay of the reference
@pytest.mark.parametrize("name", SCEN)
def test_replay_reference_walks(gpu_available, name):
    """Per-walk parity with the reference's _solveUnified run on the same Philox stream."""
    z = golden(f"replay_{name}.npz")
    sc, s = _solver_for(name, z)
    W = int(z["n_walks"])
    u, hist = s.solve(z["points"], nWalks=W, maxSteps=int(z["max_steps"]), eps=float(z["eps"]),
                      seed=int(z["seed"]), return_history=True)
    vals = np.array([w["value"] for i in range(len(z["points"])) for w in hist[i]])
    steps = np.array([w["steps"] for i in range(len(z["points"])) for w in hist[i]])
    rv, rs = z["walk_values"], z["walk_steps"]
    assert np.array_equal(steps, rs), f"step counts differ on {np.sum(steps != rs)} of {len(rs)} walks"
    scale = max(np.abs(rv).max(), 1e-30)
    close = np.abs(vals - rv) <= 1e-4 * np.abs(rv) + 1e-6 * scale
    assert close.mean() >= 0.99, _diag(vals, rv)
    np.testing.assert_allclose(vals, rv, rtol=2e-3, atol=1e-5 * scale)
    np.testing.assert_allclose(u.ravel(), z["u"], rtol=1e-4, atol=1e-6 * scale)


@pytest.mark.parametrize("name", SCEN)
def test_replay_reference_histories(gpu_available, name):
    """return_history against the reference's own history_dict on the same Philox
    stream (tests/golden/replay_*.npz, path_* / src_* / boundary_values): every
    step's point and Dirichlet/Neumann distances, every source sample point and
    contribution, the boundary terms and the running totals. A walk counts as
    matching when all its records agree (2e-3 relative for positions and
    distances, 1e-4 for contributions); >= 99% must (the chaotic
    variable-coefficient scenario: its measured floor, 97%; one walk of a
    sample smaller than 100)."""
    z = golden(f"replay_{name}.npz")
    sc, s = _solver_for(name, z)
    W = int(z["n_walks"])
    pts = z["points"]
    u, hist = s.solve(pts, nWalks=W, maxSteps=int(z["max_steps"]), eps=float(z["eps"]), seed=int(z["seed"]),
                      return_history=True)
    walks = [w for i in range(len(pts)) for w in hist[i]]
    steps = z["walk_steps"]
    assert [w["steps"] for w in walks] == list(steps)
    assert all(len(w["path"]) == w["steps"] for w in walks)
    has_src = z["src_points"].shape[0] > 0
    off = np.concatenate([[0], np.cumsum(steps)])
    # positions may drift by float rounding over hundreds of steps (Neumann hits
    # feed 1-ulp differences back into the walk): 2e-3 relative, the scale of the
    # per-walk value agreement of test_device_matches_oracle
    tol = lambda a, b: np.all(np.abs(a - b) <= 2e-3 * (1.0 + np.abs(b)))
    ok = []
    for j, w in enumerate(walks):
        a, b = off[j], off[j + 1]
        P = np.array([np.asarray(st["point"], np.float32) for st in w["path"]]).reshape(-1, 2)
        dd = np.array([st["dirichlet_distance"] for st in w["path"]], np.float32)
        dn = np.array([np.nan if st["neumann_distance"] is None else st["neumann_distance"] for st in w["path"]],
                      np.float32)
        good = tol(P, z["path_points"][a:b]) and tol(dd, z["path_dd"][a:b])
        rdn = z["path_dn"][a:b]
        good = good and np.array_equal(np.isnan(dn), np.isnan(rdn)) and np.array_equal(np.isinf(dn), np.isinf(rdn))
        fin = np.isfinite(rdn)
        good = good and tol(dn[fin], rdn[fin])
        src = [c for c in w["contributions"] if c["type"] == "source"]
        bnd = w["contributions"][-1]
        assert bnd["type"] == "boundary" and bnd["step"] == w["steps"]
        if has_src:
            assert len(src) == w["steps"]
            SP = np.array([np.asarray(c["point"], np.float32) for c in src]).reshape(-1, 2)
            SV = np.array([c["contribution"] for c in src], np.float32)
            scale = max(float(np.abs(z["src_values"]).max()), 1e-30)
            good = good and tol(SP, z["src_points"][a:b])
            good = good and np.all(np.abs(SV - z["src_values"][a:b]) <= 1e-4 * np.abs(z["src_values"][a:b]) + 1e-6 * scale)
        else:
            assert not src
        good = good and tol(np.asarray(bnd["point"], np.float32), z["final_points"][j])
        # g vanishes near the boundary of the manufactured problems: an absolute floor
        # at the walk values' scale, like the per-walk value test above
        vscale = max(float(np.abs(z["walk_values"]).max()), 1e-30)
        good = good and abs(bnd["contribution"] - z["boundary_values"][j]) <= 1e-4 * abs(z["boundary_values"][j]) + 1e-6 * vscale
        ok.append(bool(good))
    ok = np.array(ok)
    from test_oracle_golden import AGREEMENT_FLOOR   # the scenario's measured chaos (1-ulp sensitivity)
    floor = min(0.99, AGREEMENT_FLOOR.get(name, 0.99), 1.0 - 1.0 / len(ok))   # small samples: one walk
    assert ok.mean() >= floor, f"{(~ok).sum()} of {len(ok)} walks differ"
    # running point totals (:308) follow from the per-walk values
    tot = np.array([w["total_contribution"] for w in walks])
    vals = np.array([w["value"] for w in walks], np.float64)
    for i in range(len(pts)):
        np.testing.assert_allclose(tot[i * W:(i + 1) * W], np.cumsum(vals[i * W:(i + 1) * W]), rtol=1e-12)


def test_history_is_consistent_with_walk_results(gpu_available):
    """The recorder's own invariants on a larger solve: path[0] is the query point,
    each walk's value is the float32 sum of its contributions in order, and the
    recorded walks are the same walks solve_walks() returns."""
    sc, s = _solver_for("dcr_dipole")
    pts = sc.points[18:22]
    W = 256
    u, hist = s.solve(pts, nWalks=W, maxSteps=sc.max_steps, eps=sc.eps, seed=8, return_history=True)
    v, st = s.solve_walks(pts, nWalks=W, maxSteps=sc.max_steps, eps=sc.eps, seed=8)
    for i in range(len(pts)):
        for j, w in enumerate(hist[i]):
            assert w["steps"] == st[i, j] and np.float32(w["value"]) == v[i, j]
            if w["steps"]:
                np.testing.assert_array_equal(np.asarray(w["path"][0]["point"], np.float32), pts[i])
            acc = np.float32(0.0)
            for c in w["contributions"]:
                acc = np.float32(acc + np.float32(c["contribution"]))
            assert acc == v[i, j]


def _diag(got, ref):
    d = np.abs(np.asarray(got, np.float64) - np.asarray(ref, np.float64))
    rel = d / np.maximum(np.abs(ref), 1e-30)
    worst = np.argsort(-d)[:5]
    return (f"rel-diff quantiles 50/99/99.9/max: {np.quantile(rel, [0.5, 0.99, 0.999, 1.0])}; "
            f"worst: {[(int(i), float(got[i]), float(ref[i])) for i in worst]}")


# ---------------------------------------------------------------- device vs oracle
@pytest.mark.parametrize("name", SCEN)
def test_device_matches_oracle(gpu_available, name):
    """Same Philox stream, same inputs: the share of walks with identical step counts
    and values within 1e-3 must reach the scenario's floor (measured on the oracle
    itself under a 1-ulp perturbation, test_oracle_golden.AGREEMENT_FLOOR), and the
    per-point means agree to 0.5 Monte-Carlo standard errors."""
    from oracle import oracle as O
    from test_oracle_golden import AGREEMENT_FLOOR, SENS_SIZES, sensitivity_points

    sc, s = _solver_for(name)
    npts, W = SENS_SIZES[name]
    pts = sensitivity_points(sc, name, npts)
    seed = 31337
    u, st = s.solve(pts, nWalks=W, maxSteps=sc.max_steps, eps=sc.eps, seed=seed, return_stats=True)
    gv, gs = s.solve_walks(pts, nWalks=W, maxSteps=sc.max_steps, eps=sc.eps, seed=seed)
    gv, gs = gv.ravel(), gs.ravel()
    pb = O.Problem.from_scenario(sc, sigma_bar=s.sigma_bar or 0.0)
    ov, os_ = pb.solve_walks(pts, W, sc.max_steps, sc.eps, seed)
    scale = max(np.abs(ov).max(), 1e-30)
    same = (gs == os_) & (np.abs(gv - ov) <= 1e-3 * np.abs(ov) + 1e-5 * scale)
    assert same.mean() >= AGREEMENT_FLOOR[name], _diag(gv, ov)
    om = ov.astype(np.float64).reshape(npts, W).mean(1)
    ose = ov.astype(np.float64).reshape(npts, W).std(1, ddof=1) / np.sqrt(W)
    assert np.all(np.abs(st.mean - om) <= 0.5 * ose + 1e-6 * scale)


# ---------------------------------------------------------------- statistics vs the reference's own RNG
STAT_WALKS = {"laplace_square": 20000, "manufactured_polynomial": 20000, "poisson_square": 20000,
              "variable_coefficients": 20000, "dcr_dipole": 20000, "notebook_dcr": 4000,
              "wenner_topography": 20000, "wenner_topography_physical": 20000}


@pytest.mark.parametrize("name", SCEN + ["wenner_topography", "wenner_topography_physical"])
def test_statistics_vs_reference_rng(gpu_available, name):
    """Against the reference run with its OWN random streams (torch/numpy RNG): every
    reference per-point mean (n walks) is a plausible n-walk mean of the device's walks
    (bootstrap, two-sided p > 1e-3 per point); likewise the mean walk lengths. C5 (round
    5): 16 electrodes x 200 reference walks on the 10k-segment topography, both fields."""
    from test_oracle_golden import bootstrap_pvalues

    z = golden(f"stats_{name}.npz")
    sc, s = _solver_for(name)
    W = STAT_WALKS[name]
    npts = len(z["points"])
    v, st = s.solve_walks(z["points"], nWalks=W, maxSteps=int(z["max_steps"]), eps=float(z["eps"]), seed=77)
    v, st = v.astype(np.float64), st.astype(np.float64)
    p = bootstrap_pvalues(v, int(z["n_walks"]), z["mean"])
    assert p.min() > 1e-3, p
    ps = bootstrap_pvalues(st, int(z["n_walks"]), z["mean_steps"], seed=1)
    assert ps.min() > 1e-3, ps


# ---------------------------------------------------------------- determinism and sharding
def test_determinism_and_block_sharding(gpu_available):
    sc, s = _solver_for("variable_coefficients")
    pts = sc.points[:6]
    W = 10000
    nb = s.num_blocks(len(pts), W)
    full = s.solve_blocks(pts, W, 0, nb, sc.max_steps, sc.eps, seed=5)
    again = s.solve_blocks(pts, W, 0, nb, sc.max_steps, sc.eps, seed=5)
    assert np.array_equal(full, again)
    cut = [0, 1, 5, nb // 2, nb - 1, nb]
    parts = np.concatenate([s.solve_blocks(pts, W, a, b, sc.max_steps, sc.eps, seed=5) for a, b in zip(cut, cut[1:])])
    assert np.array_equal(parts, full)
    # a different seed gives different walks
    other = s.solve_blocks(pts, W, 0, nb, sc.max_steps, sc.eps, seed=6)
    assert not np.array_equal(other, full)


def test_laplace_converges_to_exact(gpu_available):
    """g = x^2 - y^2 is harmonic: the estimate converges to it (C1a, 64 x 100k walks)."""
    sc, s = _solver_for("laplace_square")
    u, st = s.solve(sc.points, nWalks=100_000, maxSteps=sc.max_steps, eps=sc.eps, seed=1, return_stats=True)
    exact = sc.points[:, 0].astype(np.float64) ** 2 - sc.points[:, 1].astype(np.float64) ** 2
    z = (st.mean - exact) / st.stderr
    # the eps-shell bias of WoS (plus quirk Q7) is O(eps) = 1e-4
    assert np.all(np.abs(st.mean - exact) < 5 * st.stderr + 3e-4)
    assert np.sqrt(np.mean(z ** 2)) < 3.0


@pytest.mark.parametrize("name", SCEN)
def test_jit_kernel_matches_interpreted_kernel(gpu_available, name):
    """The hiprtc field-specialised walk kernel and the precompiled kernel that
    interprets the field program give bit-identical per-walk results."""
    sc, s = _solver_for(name)
    pts = sc.points[:8]
    W = 2048
    v1, s1 = s.solve_walks(pts, nWalks=W, maxSteps=sc.max_steps, eps=sc.eps, seed=3)
    assert s.last_timing["jit"] == 1, "the field-specialised kernel did not build"
    s.set_jit(False)
    v0, s0 = s.solve_walks(pts, nWalks=W, maxSteps=sc.max_steps, eps=sc.eps, seed=3)
    assert s.last_timing["jit"] == 0
    assert np.array_equal(s1, s0)
    assert np.array_equal(v1.view(np.uint32), v0.view(np.uint32)) or np.array_equal(v1, v0)


# ---------------------------------------------------------------- full-size properties
def test_dcr_full_size_linearity(gpu_available):
    """C4 at its full size (48 electrodes x 1M walks): the walk does not depend on the
    source, so doubling f doubles every contribution exactly (power of two): u(2f)
    must equal 2 u(f) bit for bit, and the step totals must be identical."""
    from dcrmontecarlo_amd import scenarios as S
    from dcrmontecarlo_amd.geometry import PolyLinesSimple
    from dcrmontecarlo_amd.solvers import WostSolver_2D

    sc = S.dcr_dipole()
    mk = lambda f: WostSolver_2D(PolyLinesSimple(sc.dirichlet), sc.g, PolyLinesSimple(sc.neumann), source=f,
                                 alpha=sc.alpha)
    s1, s2 = mk(sc.f), mk(2.0 * sc.f)
    u1, st1 = s1.solve(sc.points, nWalks=sc.n_walks, maxSteps=sc.max_steps, eps=sc.eps, seed=9, return_stats=True)
    u2, st2 = s2.solve(sc.points, nWalks=sc.n_walks, maxSteps=sc.max_steps, eps=sc.eps, seed=9, return_stats=True)
    assert np.all(np.isfinite(st1.mean))
    assert np.array_equal(st2.mean, 2.0 * st1.mean)
    assert st1.total_steps == st2.total_steps
    assert st1.total_steps > 48 * 1_000_000 * 20
    assert np.all(st1.mean_steps > 1)


def test_variable_coefficients_full_size_homogeneity(gpu_available):
    """C3 at its BASELINE size (configs[2]: 256 points x 100k walks, delta tracking and
    the Neumann circle): the walks depend only on alpha and sigma, so doubling both the
    boundary values g and the source f doubles every walk's total exactly (a power of
    two): u(2g, 2f) must equal 2 u(g, f) bit for bit with identical step totals, and
    the solve is deterministic."""
    from dcrmontecarlo_amd import scenarios as S
    from dcrmontecarlo_amd.geometry import PolyLinesSimple
    from dcrmontecarlo_amd.solvers import WostSolver_2D

    sc = S.variable_coefficients()
    assert sc.points.shape[0] == 256 and sc.n_walks == 100_000
    mk = lambda k: WostSolver_2D(PolyLinesSimple(sc.dirichlet), k * sc.g, PolyLinesSimple(sc.neumann),
                                 source=k * sc.f, sigma=sc.sigma, alpha=sc.alpha)
    s1, s2 = mk(1.0), mk(2.0)
    assert s1.sigma_bar == s2.sigma_bar
    kw = dict(nWalks=sc.n_walks, maxSteps=sc.max_steps, eps=sc.eps, seed=12, return_stats=True)
    u1, st1 = s1.solve(sc.points, **kw)
    u1b, st1b = s1.solve(sc.points, **kw)
    u2, st2 = s2.solve(sc.points, **kw)
    assert np.all(np.isfinite(st1.mean))
    assert np.array_equal(st1.mean, st1b.mean) and st1.total_steps == st1b.total_steps
    assert np.array_equal(st2.mean, 2.0 * st1.mean)
    assert st1.total_steps == st2.total_steps
    assert st1.total_steps > 256 * 100_000 * 10


# ---------------------------------------------------------------- edge cases
def test_edge_cases(gpu_available):
    from dcrmontecarlo_amd import fields as F
    from dcrmontecarlo_amd.geometry import PolyLinesSimple
    from dcrmontecarlo_amd.solvers import WostSolver_2D

    sq = PolyLinesSimple(np.array([[0, 0], [1, 0], [1, 1], [0, 1], [0, 0]], np.float32))
    s = WostSolver_2D(sq, F.X + 2 * F.Y)
    p = np.array([[0.25, 0.5]], np.float32)
    # eps >= 1: dDirichlet is seeded with 1.0, no step is taken, u = g(x0) (quirk Q12)
    u, st = s.solve(p, nWalks=10, eps=1.0, return_stats=True)
    assert u[0, 0] == pytest.approx(1.25) and st.total_steps == 0
    # maxSteps = 0: likewise
    u, st = s.solve(p, nWalks=10, maxSteps=0, return_stats=True)
    assert u[0, 0] == pytest.approx(1.25) and st.total_steps == 0
    # one walk, many points, ragged point counts
    u = s.solve(np.random.default_rng(0).uniform(0.1, 0.9, (1001, 2)).astype(np.float32), nWalks=1)
    assert u.shape == (1001, 1) and np.all(np.isfinite(u))
    # empty point set
    assert s.solve(np.zeros((0, 2), np.float32), nWalks=4).shape == (0, 1)
    # walks_per_point not a multiple of the block size
    u1, st1 = s.solve(p, nWalks=4097, seed=3, return_stats=True)
    assert st1.walks == 4097
    # a zero-length segment makes the reference's distance NaN (0/0, PolylinesSimple.py:43)
    deg = PolyLinesSimple(np.array([[0, 0], [1, 0], [1, 0], [1, 1], [0, 1], [0, 0]], np.float32))
    assert np.isnan(deg.distance(np.array([0.5, 0.5], np.float32)))
    # torch in -> torch out, like the reference
    torch = pytest.importorskip("torch")
    ut = s.solve(torch.tensor([[0.5, 0.5]]), nWalks=16)
    assert isinstance(ut, torch.Tensor) and ut.shape == (1, 1) and ut.dtype == torch.float32
    # invalid arguments fail loudly
    with pytest.raises(ValueError):
        s.solve(p, nWalks=0)
    with pytest.raises(ValueError):
        WostSolver_2D(sq, F.X, alpha=F.X + 2).solve(p, nWalks=4)   # delta tracking without a source (Q14)
    with pytest.raises(ValueError):             # unknown compat mode
        WostSolver_2D(sq, F.X, source=1.0, sigma=1.0, compat="corrected")
