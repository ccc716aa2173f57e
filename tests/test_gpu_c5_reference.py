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


@pytest.mark.parametrize("name", ["wenner_topography", "wenner_topography_physical"])
def test_c5_replay_reference_histories(gpu_available, name):
    """return_history on C5 against the reference's own history_dict on the same Philox
    stream (tests/golden/replay_<name>.npz: 8 electrodes x 32 walks on the 10k-segment
    topography, solvers/WoStSolver.py:184-309, structure :335-349): every step's point and
    Dirichlet / silhouette distances, every source sample point and contribution and the
    boundary term. A walk matches when its step count is the reference's and all its
    records agree (2e-3 relative for points and distances, 1e-4 for contributions, as
    tests/test_gpu_parity.py); the matching share must reach the oracle's own agreement
    with the reference on these walks (its per-walk floor, measured here) less 0.02. Each
    diverged walk's first divergent step is classified and printed."""
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
    scale = max(float(np.abs(z["src_values"]).max()), 1e-30)
    vscale = max(float(np.abs(z["walk_values"]).max()), 1e-30)
    tol = lambda x, y: bool(np.all(np.abs(x - y) <= 2e-3 * (1.0 + np.abs(y))))
    ok, kinds = [], Counter()
    for j, w in enumerate(walks):
        P = np.array([np.asarray(st["point"], np.float32) for st in w["path"]]).reshape(-1, 2)
        DD = np.array([st["dirichlet_distance"] for st in w["path"]], np.float32)
        DN = np.array([np.nan if st["neumann_distance"] is None else st["neumann_distance"] for st in w["path"]],
                      np.float32)
        src = [c for c in w["contributions"] if c["type"] == "source"]
        assert len(src) == w["steps"] and len(w["path"]) == w["steps"]
        SP = np.array([np.asarray(c["point"], np.float32) for c in src]).reshape(-1, 2)
        SV = np.array([c["contribution"] for c in src], np.float32)
        bnd = w["contributions"][-1]
        assert bnd["type"] == "boundary" and bnd["step"] == w["steps"]
        a, b = off[j], off[j + 1]
        good = w["steps"] == rs[j]
        if good:
            rdn = z["path_dn"][a:b]
            fin = np.isfinite(rdn)
            good = (tol(P, z["path_points"][a:b]) and tol(DD, z["path_dd"][a:b])
                    and np.array_equal(np.isnan(DN), np.isnan(rdn)) and tol(DN[fin], rdn[fin])
                    and tol(SP, z["src_points"][a:b])
                    and bool(np.all(np.abs(SV - z["src_values"][a:b]) <= 1e-4 * np.abs(z["src_values"][a:b])
                                    + 1e-6 * scale))
                    and tol(np.asarray(bnd["point"], np.float32), z["final_points"][j])
                    and abs(bnd["contribution"] - z["boundary_values"][j])
                    <= 1e-4 * abs(z["boundary_values"][j]) + 1e-6 * vscale)
        if not good:
            kinds[_first_divergence(w, z, a, min(int(rs[j]), int(w["steps"])), (P, DD, DN, SP))] += 1
        ok.append(bool(good))
    ok = np.array(ok)
    pb = O.Problem(z["dirichlet"], z["neumann"], sc.g, sc.f, sc.sigma, sc.alpha)
    pb = O.Problem(z["dirichlet"], z["neumann"], sc.g, sc.f, sc.sigma, sc.alpha, sigma_bar=pb.sigma_bar())
    ov, os_ = pb.solve_walks(pts, W, kw["maxSteps"], kw["eps"], kw["seed"])
    o_same, _ = c5_replay_agreement(ov, os_, z)
    print(f"{name}: {ok.mean():.4f} of {len(ok)} walk histories match the reference's (the oracle's walks "
          f"{o_same:.4f}); first divergence of the others: {dict(kinds)}")
    assert ok.mean() >= o_same - 0.02, (ok.mean(), o_same, dict(kinds))


def test_c5_device_replays_reference_rho_a(gpu_available):
    """G13: the reference's own C5 Wenner survey (setSourceTerm + _solveUnified on the
    Philox stream, physical conductivity and background, 16 quadripoles x both receivers x
    64 walks; tests/golden/rho_replay_wenner_topography_physical.npz) against the device on
    the same walks, launched per electrode group as run_wenner_survey launches them: the
    walks identical at least as often as the oracle's (0.980 on all 16 quadripoles) less
    0.02, and every quadripole's dV and rho_a within the bound its diverged walks allow
    (survey.compare_wenner_replay)."""
    import os

    from dcrmontecarlo_amd import scenarios as S
    from dcrmontecarlo_amd import survey as SV

    ref = SV.load_wenner_replay(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden",
                                             "rho_replay_wenner_topography_physical.npz"))
    sc = S.wenner_topography_physical(n_walks=1)
    sm = sc.solver(device=0)
    sh = SV.homogeneous_solver(sc, ref.alpha_bg, sm, device=0)
    out = SV.compare_wenner_replay(*SV.wenner_replay_walks(ref, SV.solver_replay_walks(sm, sh, ref)), ref)
    print("C5 rho_a replay: walks identical", out["walks_identical"], "diverged per quadripole",
          out["diverged_walks"], "dV max d/sigma_chaos", out["dv_model"]["max_d_over_sigma_chaos"])
    assert out["walks_identical"] >= 0.96, out["walks_identical"]
    assert out["all_within_tolerance"], out
