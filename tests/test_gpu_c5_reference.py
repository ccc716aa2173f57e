"""C5 on the device against the reference's own outputs (tools/gen_fixtures.py; see
tests/test_c5_reference.py for the fixtures and the tolerances' origin):

* sigma_bar and sigma' of both C5 variants equal the reference's (solvers/WoStSolver.py:
  37-43, 66-138 with utils.py:65-120): sigma_bar within 1e-5 relative;
* the segment tree on the device (wost_geometry_query(op | WOST_GEOM_TREE)) returns the
  reference's silhouette distances and intersections at 320 recorded C5 walk positions,
  and the device's full scans bit for bit;
* the reference's C5 walks replayed on the Philox stream (8 electrodes x 32 walks):
  the device's walks (tree kernel, field-specialised) agree at least as often as the
  oracle agrees with itself under a 1-ulp change of the step direction, less 2 points,
  >= 95% of the walk values are within 1e-4, and the per-electrode means agree within
  3 combined standard errors.
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
    same, close = c5_replay_agreement(v.ravel(), st.ravel(), z)
    # the oracle's own 1-ulp chaos on the same walks (its own sigma_bar)
    pb = O.Problem(z["dirichlet"], z["neumann"], sc.g, sc.f, sc.sigma, sc.alpha)
    pb = O.Problem(z["dirichlet"], z["neumann"], sc.g, sc.f, sc.sigma, sc.alpha, sigma_bar=pb.sigma_bar())
    args = (z["points"], W, int(z["max_steps"]), float(z["eps"]), int(z["seed"]))
    ov, os_ = pb.solve_walks(*args)
    try:
        O.set_direction_perturbation(1.2e-7)
        pv, ps = pb.solve_walks(*args)
    finally:
        O.set_direction_perturbation(0.0)
    scale = max(float(np.abs(ov).max()), 1e-30)
    chaos = float(((ps == os_) & (np.abs(pv - ov) <= 1e-3 * np.abs(ov) + 1e-5 * scale)).mean())
    assert same >= chaos - 0.02, (same, chaos)
    assert close >= 0.95, close
    # per-electrode means within 3 combined standard errors: a walk that diverged (chaos)
    # carries a heavy-tailed value of the literal fields, so exact means are not expected
    n = len(z["points"])
    g = v.astype(np.float64).reshape(n, -1)
    r = z["walk_values"].reshape(n, -1)
    se = np.sqrt(g.var(1, ddof=1) / W + r.var(1, ddof=1) / W)
    assert np.all(np.abs(g.mean(1) - r.mean(1)) <= 3.0 * se + 1e-9 * np.abs(r).max()), (g.mean(1), r.mean(1), se)
