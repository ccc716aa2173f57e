"""C5 on the device against the reference's own outputs (tools/gen_fixtures.py; see
tests/test_c5_reference.py for the fixtures and the tolerances' origin):

* sigma_bar and sigma' of both C5 variants equal the reference's (solvers/WoStSolver.py:
  37-43, 66-138 with utils.py:65-120): sigma_bar within 1e-5 relative;
* the segment tree on the device (wost_geometry_query(op | WOST_GEOM_TREE)) returns the
  reference's silhouette distances and intersections at 320 recorded C5 walk positions,
  and the device's full scans bit for bit;
* the reference's C5 walks replayed on the Philox stream (8 electrodes x 32 walks):
  the device's walks (tree kernel, field-specialised) are the oracle's and agree with
  the reference's as often as the oracle's do (less 0.02), >= 95% of the walk values
  are within 1e-4, and the per-electrode means agree within 1e-3;
* G13: the reference's C5 Wenner survey (physical fields) replayed on the same walks:
  every quadripole's dV and rho_a within the bound its diverged walks allow.
"""
import numpy as np
import pytest

from conftest import golden
from test_c5_reference import K, c5_replay_agreement, check_against_reference_kats

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["wenner_topography", "wenner_topography_physical"])
def test_c5_sigma_bar_and_fields_device(gpu_available, name):
    from dcrmontecarlo_amd import scenarios as S

    z = golden(f"fields_{name}.npz")
    sc = S.ALL[name](n_walks=1)
    s = sc.solver(device=0)
    assert s.use_delta_tracking
    assert s.sigma_bar == pytest.approx(float(z["sigma_bar"]), rel=1e-5)
    P = z["points"]
    for key in ("f", "alpha"):
        ref = z[key]
        got = s.eval_field(key, P)[:, 0].astype(np.float64)
        np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-6 * max(np.abs(ref).max(), 1e-30), err_msg=key)
    sp = s.eval_field("sigma_prime", P)[:, 0].astype(np.float64)
    ref = z["sigma_prime"]
    fin = np.isfinite(ref)
    np.testing.assert_allclose(sp[fin], ref[fin], rtol=2e-3, atol=1e-5 * np.abs(ref[fin]).max())


def test_c5_device_tree_queries_reproduce_reference_kats(gpu_available):
    from dcrmontecarlo_amd.geometry import PolyLinesSimple

    z = golden("geometry_kats_c5.npz")
    V, P, D, R = (z[K + k] for k in ("verts", "points", "dirs", "radii"))
    poly = PolyLinesSimple(V)
    sil_t = poly.silhouetteDistance(P, tree=True)
    hp, nrm, found = poly.intersectPolylines(P, D, R, tree=True)
    hit_t = np.concatenate([hp, nrm, found[:, None].astype(np.float32)], axis=1).astype(np.float32)
    check_against_reference_kats(sil_t, hit_t, z, "device tree")
    # and the device's own full scans, bit for bit
    sil_s = poly.silhouetteDistance(P)
    hp, nrm, found = poly.intersectPolylines(P, D, R)
    hit_s = np.concatenate([hp, nrm, found[:, None].astype(np.float32)], axis=1).astype(np.float32)
    np.testing.assert_array_equal(sil_t.view(np.uint32), sil_s.view(np.uint32))
    np.testing.assert_array_equal(hit_t.view(np.uint32), hit_s.view(np.uint32))


def test_c5_device_tree_queries_refuse_other_ops(gpu_available):
    from dcrmontecarlo_amd.geometry import PolyLinesSimple

    poly = PolyLinesSimple(np.array([[0, 0], [1, 0]], np.float32))
    with pytest.raises(ValueError):
        poly.silhouetteDistance(np.zeros((4, 2), np.float32), tree=True)   # one segment: no tree


def test_c5_device_replays_reference_walks(gpu_available):
    """The reference's C5 walks on the Philox stream, the device's tree kernel with its
    own sigma_bar and the default trig (wost_set_trig AUTO: correctly rounded directions
    on this curved boundary; the segment angles from the C library's atan2f, as torch's).
    Round 4's device left the reference's path at the first step of every walk (hardware
    v_sin/v_cos, the device's atan2f on half of the segments: tools/r05/c5_divergence.py)
    and kept 82% of the walks; now its walks are the oracle's (>= 99% identical) and it
    keeps as many of the reference's as the oracle does (0.930, the remaining 7% the
    reference's own MKL cos/sin ulps and 10k-element torch reductions). Per-electrode
    means within 1e-3 as the oracle's (tests/test_c5_reference.py)."""
    from oracle import oracle as O

    from dcrmontecarlo_amd import scenarios as S
    from dcrmontecarlo_amd.geometry import PolyLinesSimple
    from dcrmontecarlo_amd.solvers import WostSolver_2D

    z = golden("replay_wenner_topography.npz")
    sc = S.wenner_topography(n_walks=1)
    s = WostSolver_2D(PolyLinesSimple(z["dirichlet"]), sc.g, PolyLinesSimple(z["neumann"]), source=sc.f,
                      alpha=sc.alpha)
    assert s.sigma_bar == pytest.approx(float(z["sigma_bar"]), rel=1e-5)
    W = int(z["n_walks"])
    v, st = s.solve_walks(z["points"], nWalks=W, maxSteps=int(z["max_steps"]), eps=float(z["eps"]),
                          seed=int(z["seed"]))
    assert s.last_timing["tree"] == 1
    v, st = v.ravel(), st.ravel()
    same, close = c5_replay_agreement(v, st, z)
    pb = O.Problem(z["dirichlet"], z["neumann"], sc.g, sc.f, sc.sigma, sc.alpha)
    pb = O.Problem(z["dirichlet"], z["neumann"], sc.g, sc.f, sc.sigma, sc.alpha, sigma_bar=pb.sigma_bar())
    ov, os_ = pb.solve_walks(z["points"], W, int(z["max_steps"]), float(z["eps"]), int(z["seed"]))
    o_same, _ = c5_replay_agreement(ov, os_, z)
    scale = max(float(np.abs(ov).max()), 1e-30)
    dev_oracle = float(((st == os_) & (np.abs(v - ov) <= 1e-3 * np.abs(ov) + 1e-5 * scale)).mean())
    print(f"C5 replay: device walks identical to the reference's {same:.4f} (oracle {o_same:.4f}), "
          f"to the oracle's {dev_oracle:.4f}")
    assert dev_oracle >= 0.99, dev_oracle
    assert same >= o_same - 0.02 and same >= 0.906 - 0.02, (same, o_same)
    assert close >= 0.95, close
    n = len(z["points"])
    m_g = v.astype(np.float64).reshape(n, -1).mean(1)
    m_r = z["walk_values"].reshape(n, -1).mean(1)
    np.testing.assert_allclose(m_g, m_r, rtol=1e-3, atol=1e-6 * np.abs(m_r).max())


def _first_divergence(hist_w, z, a, n, rec):
    """Where one diverged walk first leaves the reference's replayed path (tools/r05/
    c5_divergence.py's classes): the first step j whose point or query distances differ,
    classified by the transition j-1 -> j -- distance (the queries at j-1 differ),
    direction (the source sample point at j-1 differs: direction or radius), collision
    (same sample point, one walk moved to it and the other to the ray's point), ray (both
    moved to the ray's point, which differs: the hit test) -- or `end` when every common
    step agrees (step count or boundary term)."""
    P, DD, DN, SP = rec
    tol = lambda x, y: np.abs(x - y) <= 2e-3 * (1.0 + np.abs(y))
    RP, Rd, Rn, RS = (z[k][a:a + n] for k in ("path_points", "path_dd", "path_dn", "src_points"))
    GP, Gd, Gn, GS = P[:n], DD[:n], DN[:n], SP[:n]
    dn_ok = (np.isnan(Gn) == np.isnan(Rn)) & np.where(np.isfinite(Rn), tol(Gn, np.nan_to_num(Rn)), True)
    bad = ~(tol(GP, RP).all(1) & tol(Gd, Rd) & dn_ok)
    if not bad.any():
        return "end"
    j = int(np.argmax(bad))
    if j == 0:
        return "start"
    i = j - 1
    if not (tol(Gd[i], Rd[i]) and dn_ok[i]):
        return "distance"
    if not tol(GS[i], RS[i]).all():
        return "direction"
    r_col, g_col = bool(np.all(RP[j] == RS[i])), bool(np.all(GP[j] == GS[i]))
    return "collision" if r_col != g_col else ("sample" if r_col else "ray")


def _history_agreement(P, SP, steps, z, tol_rel=2e-3):
    """(share of the reference's step records a history reproduces before its first
    divergence, share of walks whose whole history agrees): a walk's records agree while
    its pre-step point and source sample point stay within tol_rel of the reference's.
    P, SP: per walk [steps, 2] arrays."""
    rs = np.asarray(z["walk_steps"], np.int64)
    ro = np.concatenate([[0], np.cumsum(rs)])
    tol = lambda x, y: np.all(np.abs(x - y) <= tol_rel * (1.0 + np.abs(y)), axis=1)
    pre = full = 0
    for w in range(len(rs)):
        n = min(int(rs[w]), int(steps[w]))
        ok = tol(P[w][:n], z["path_points"][ro[w]:ro[w] + n]) & tol(SP[w][:n], z["src_points"][ro[w]:ro[w] + n])
        j = n if ok.all() else int(np.argmin(ok))
        pre += j
        full += int(j == rs[w] and steps[w] == rs[w])
    return pre / float(ro[-1]), full / float(len(rs))


@pytest.mark.parametrize("name", ["wenner_topography", "wenner_topography_physical"])
def test_c5_replay_reference_histories(gpu_available, name):
    """return_history on C5 against the reference's own history_dict on the same Philox
    stream (tests/golden/replay_<name>.npz: 8 electrodes x 32 walks on the 10k-segment
    topography; solvers/WoStSolver.py:184-309, structure :335-349).

    C5's walks are chaotic: the reference's own last-ulp arithmetic (torch's MKL cos/sin,
    its 10k-element reductions) sends a walk off its replayed path at some step, and the
    divergence grows -- so the walk values agree far more often (0.93 literal, of which
    more than half are 0: weights that underflow in the literal fields' 'air') than whole
    histories do (0.34 literal, 0.82 physical). The floor is therefore the oracle's OWN
    history agreement with the reference on the same walks, measured here with its
    recorder (oracle orc_solve_history): the device's histories must reproduce as many of
    the reference's step records before their first divergence, and as many whole walks,
    as the oracle's, less 0.02; and reproduce >= 97% of the oracle's own records before
    their walks' first divergence. Each walk's records have the reference's structure; the walks whose
    whole path agrees carry the reference's source contributions (1e-3 relative: the
    weights' float rounding accumulates over ~200 steps) and boundary terms; the first
    divergence of the other walks is classified and printed."""
    from collections import Counter

    from oracle import oracle as O

    from dcrmontecarlo_amd import scenarios as S
    from dcrmontecarlo_amd.geometry import PolyLinesSimple
    from dcrmontecarlo_amd.solvers import WostSolver_2D

    z = golden(f"replay_{name}.npz")
    sc = S.ALL[name](n_walks=1)
    s = WostSolver_2D(PolyLinesSimple(z["dirichlet"]), sc.g, PolyLinesSimple(z["neumann"]), source=sc.f,
                      alpha=sc.alpha)
    W, pts = int(z["n_walks"]), z["points"]
    kw = dict(maxSteps=int(z["max_steps"]), eps=float(z["eps"]), seed=int(z["seed"]))
    u, hist = s.solve(pts, nWalks=W, return_history=True, **kw)
    assert s.last_timing["tree"] == 1
    walks = [w for i in range(len(pts)) for w in hist[i]]
    rs = z["walk_steps"]
    off = np.concatenate([[0], np.cumsum(rs)])
    P, DD, DN, SP, SV, steps = [], [], [], [], [], []
    for w in walks:   # the reference's structure (:197-309)
        assert len(w["path"]) == w["steps"]
        src = [c for c in w["contributions"] if c["type"] == "source"]
        assert len(src) == w["steps"] and [c["step"] for c in src] == list(range(w["steps"]))
        bnd = w["contributions"][-1]
        assert bnd["type"] == "boundary" and bnd["step"] == w["steps"]
        P.append(np.array([np.asarray(st["point"], np.float32) for st in w["path"]]).reshape(-1, 2))
        DD.append(np.array([st["dirichlet_distance"] for st in w["path"]], np.float32))
        DN.append(np.array([np.nan if st["neumann_distance"] is None else st["neumann_distance"]
                            for st in w["path"]], np.float32))
        SP.append(np.array([np.asarray(c["point"], np.float32) for c in src]).reshape(-1, 2))
        SV.append(np.array([c["contribution"] for c in src], np.float32))
        steps.append(w["steps"])
    steps = np.array(steps)
    pb = O.Problem(z["dirichlet"], z["neumann"], sc.g, sc.f, sc.sigma, sc.alpha)
    pb = O.Problem(z["dirichlet"], z["neumann"], sc.g, sc.f, sc.sigma, sc.alpha, sigma_bar=pb.sigma_bar())
    ov, os_, orec = pb.solve_history(pts, W, kw["maxSteps"], kw["eps"], kw["seed"])
    # the device's histories are the oracle's: its share of the oracle's records before each
    # walk's first divergence (the device's sampler table differs from the oracle's by <= 2e-6,
    # test_sampler_table_vs_oracle, and an ulp in a sampled radius drifts a few long walks
    # apart near their ends: 0.980 literal, 0.9996 physical measured)
    zo = {"walk_steps": os_, "path_points": np.concatenate([orec[w, :os_[w], :2] for w in range(len(os_))]),
          "src_points": np.concatenate([orec[w, :os_[w], 2:] for w in range(len(os_))])}
    dev_oracle, _ = _history_agreement(P, SP, steps, zo)
    d_pre, d_full = _history_agreement(P, SP, steps, z)
    o_pre, o_full = _history_agreement([orec[w, :os_[w], :2] for w in range(len(os_))],
                                       [orec[w, :os_[w], 2:] for w in range(len(os_))], os_, z)
    # the walks whose whole path agrees: their contributions and boundary terms
    tol = lambda x, y: bool(np.all(np.abs(x - y) <= 2e-3 * (1.0 + np.abs(y))))
    scale = max(float(np.abs(z["src_values"]).max()), 1e-30)
    vscale = max(float(np.abs(z["walk_values"]).max()), 1e-30)
    kinds, bad_terms = Counter(), 0
    for j, w in enumerate(walks):
        a, b = off[j], off[j + 1]
        n = min(int(rs[j]), int(steps[j]))
        whole = (steps[j] == rs[j] and tol(P[j], z["path_points"][a:b]) and tol(SP[j], z["src_points"][a:b])
                 and tol(np.asarray(w["contributions"][-1]["point"], np.float32), z["final_points"][j]))
        if not whole:
            kinds[_first_divergence(w, z, a, n, (P[j], DD[j], DN[j], SP[j]))] += 1
            continue
        rdn = z["path_dn"][a:b]
        fin = np.isfinite(rdn)
        # a distance moves no more than its point (1-Lipschitz): the points' own slack added
        slack = np.abs(P[j] - z["path_points"][a:b]).sum(1)
        ok = (bool(np.all(np.abs(DD[j] - z["path_dd"][a:b]) <= 2e-3 * (1.0 + np.abs(z["path_dd"][a:b])) + slack))
              and np.array_equal(np.isnan(DN[j]), np.isnan(rdn))
              and bool(np.all(np.abs(DN[j][fin] - rdn[fin]) <= 2e-3 * (1.0 + np.abs(rdn[fin])) + slack[fin]))
              and bool(np.all(np.abs(SV[j] - z["src_values"][a:b]) <= 1e-3 * np.abs(z["src_values"][a:b]) + 1e-6 * scale))
              and abs(w["contributions"][-1]["contribution"] - z["boundary_values"][j])
              <= 1e-3 * abs(z["boundary_values"][j]) + 1e-6 * vscale)
        bad_terms += int(not ok)
    print(f"{name}: the oracle's step records the device reproduces {dev_oracle:.4f}; the reference's step records "
          f"reproduced before the first divergence: device {d_pre:.4f}, oracle {o_pre:.4f}; whole histories: device "
          f"{d_full:.4f}, oracle {o_full:.4f}; first divergence of the others: {dict(kinds)}; whole-path walks with "
          f"other terms: {bad_terms}")
    assert dev_oracle >= 0.97, dev_oracle
    assert d_pre >= o_pre - 0.02 and d_full >= o_full - 0.02, (d_pre, o_pre, d_full, o_full)
    assert bad_terms <= max(1, int(0.02 * len(walks))), bad_terms


@pytest.mark.parametrize("name", ["wenner_topography", "wenner_topography_physical"])
def test_c5_device_replays_reference_rho_a(gpu_available, name):
    """G13: the reference's own C5 Wenner survey (setSourceTerm + _solveUnified on the
    Philox stream, model + homogeneous background, 32 quadripoles x both receivers x 64
    walks; tests/golden/rho_replay_<name>.npz -- the physical survey, and since round 6 the
    literal one the bench times) against the device on the same walks, launched per
    electrode group as run_wenner_survey launches them: the walks identical at least as
    often as the oracle's on the whole fixture (test_c5_reference.ORACLE_RHO_IDENTICAL:
    0.918 literal, 0.982 physical) less 0.02, and every quadripole's dV and rho_a within
    the bound its diverged walks allow (survey.compare_wenner_replay)."""
    import os

    from test_c5_reference import ORACLE_RHO_IDENTICAL

    from dcrmontecarlo_amd import scenarios as S
    from dcrmontecarlo_amd import survey as SV

    ref = SV.load_wenner_replay(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden",
                                             f"rho_replay_{name}.npz"))
    sc = S.ALL[name](n_walks=1)
    sm = sc.solver(device=0)
    sh = SV.homogeneous_solver(sc, ref.alpha_bg, sm, device=0)
    out = SV.compare_wenner_replay(*SV.wenner_replay_walks(ref, SV.solver_replay_walks(sm, sh, ref)), ref)
    print(f"C5 {name} rho_a replay: walks identical", out["walks_identical"], "(oracle", ORACLE_RHO_IDENTICAL[name],
          ") diverged per quadripole", out["diverged_walks"], "rho_a max d/sigma_chaos",
          out["rho_a"]["max_d_over_sigma_chaos"])
    assert out["walks_identical"] >= ORACLE_RHO_IDENTICAL[name] - 0.02, out["walks_identical"]
    assert out["all_within_tolerance"], out
