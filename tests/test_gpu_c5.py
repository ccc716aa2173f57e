"""C5 at its BASELINE configuration: the 10,000-segment topography (SURVEY 8d C5,
notebook cells 17-18 fields and U boundary) with the 256-electrode line, walked
through the segment tree, against the reference's brute-force scans restated by
the CPU oracle (geometry/PolylinesSimple.py:25-49, :83-102, :134-197).

* every step of recorded device walks: the Dirichlet distance and the Neumann
  silhouette distance the tree kernel used equal the oracle's full scans bit for
  bit (the tree must not change a single query);
* device vs oracle on the same Philox streams (32 electrodes x 512 walks): since
  round 5's correctly rounded directions the device draws the oracle's walks, so
  >= 99% of them must be identical (round 4's 0.82 fails), with the oracle's chaos
  under a 1-ulp perturbation of the step direction (~87%, the Q1 Neumann "hits")
  printed beside it; and per-electrode means within 1e-3 relative;
* full size (256 electrodes x 10k walks): u(2f) = 2 u(f) bit for bit, and the tree
  kernel equals the brute-force scan kernel walk for walk on 64 electrodes x 256
  walks (~3.4M steps through both kernels);
* the Wenner survey's multi-source batching equals per-source solves bit for bit.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu



def _c5(**kw):
    from dcrmontecarlo_amd import scenarios as S

    return S.wenner_topography(**kw)


def test_c5_tree_queries_along_walks_match_full_scans(gpu_available):
    from oracle import oracle as O

    sc = _c5()
    s = sc.solver(device=0)
    pts = sc.points[4::32]
    u, hist = s.solve(pts, nWalks=24, maxSteps=sc.max_steps, eps=sc.eps, seed=17, return_history=True)
    assert s.last_timing["tree"] == 1
    P, DD, DN = [], [], []
    for i in range(len(pts)):
        for w in hist[i]:
            for st in w["path"]:
                P.append(np.asarray(st["point"], np.float32))
                DD.append(st["dirichlet_distance"])
                DN.append(st["neumann_distance"])
    P = np.array(P, np.float32)
    DD, DN = np.array(DD, np.float32), np.array(DN, np.float32)
    assert len(P) > 10000
    dd_o = O.geometry("distance", sc.dirichlet, P)
    dn_o = O.geometry("silhouetteDistance", sc.neumann, P)
    np.testing.assert_array_equal(DD.view(np.uint32), dd_o.view(np.uint32))
    np.testing.assert_array_equal(DN.view(np.uint32), dn_o.view(np.uint32))
    assert np.isfinite(DN).sum() > 100          # silhouettes were found along the walks


def test_c5_device_matches_oracle(gpu_available):
    from oracle import oracle as O

    sc = _c5()
    s = sc.solver(device=0)
    pts = sc.points[4::8][:32]
    W = 512
    gv, gs = s.solve_walks(pts, nWalks=W, maxSteps=sc.max_steps, eps=sc.eps, seed=31337)
    gv, gs = gv.ravel(), gs.ravel()
    sb = O.Problem.from_scenario(sc).sigma_bar()        # the oracle's OWN sigma_bar (gridSampleMinMax restated)
    assert s.sigma_bar == pytest.approx(sb, rel=1e-5)
    pb = O.Problem.from_scenario(sc, sigma_bar=sb)
    ov, os_ = pb.solve_walks(pts, W, sc.max_steps, sc.eps, 31337)
    try:
        O.set_direction_perturbation(1.2e-7)       # 1 ulp of the step direction
        pv, ps = pb.solve_walks(pts, W, sc.max_steps, sc.eps, 31337)
    finally:
        O.set_direction_perturbation(0.0)
    scale = max(float(np.abs(ov).max()), 1e-30)
    agree = lambda v, st: (st == os_) & (np.abs(v - ov) <= 1e-3 * np.abs(ov) + 1e-5 * scale)
    chaos = agree(pv, ps).mean()                   # the oracle against itself, 1 ulp apart
    device = agree(gv, gs).mean()
    print(f"C5 device vs oracle: {device:.4f} of the walks identical (the oracle's 1-ulp chaos {chaos:.4f})")
    assert chaos > 0.5 and device >= 0.99, (device, chaos)
    g = gv.astype(np.float64).reshape(len(pts), W)
    o = ov.astype(np.float64).reshape(len(pts), W)
    np.testing.assert_allclose(g.mean(1), o.mean(1), rtol=1e-3, atol=1e-6 * scale)


def test_c5_full_size_linearity_and_tree_equals_scan(gpu_available):
    from dcrmontecarlo_amd.geometry import PolyLinesSimple
    from dcrmontecarlo_amd.solvers import WostSolver_2D

    sc = _c5(n_electrodes=256, n_walks=10_000)
    mk = lambda f: WostSolver_2D(PolyLinesSimple(sc.dirichlet), sc.g, PolyLinesSimple(sc.neumann), source=f,
                                 alpha=sc.alpha)
    s1, s2 = mk(sc.f), mk(2.0 * sc.f)
    u1, st1 = s1.solve(sc.points, nWalks=sc.n_walks, maxSteps=sc.max_steps, eps=sc.eps, seed=21, return_stats=True)
    assert s1.last_timing["tree"] == 1
    u2, st2 = s2.solve(sc.points, nWalks=sc.n_walks, maxSteps=sc.max_steps, eps=sc.eps, seed=21, return_stats=True)
    assert np.all(np.isfinite(st1.mean))
    assert np.array_equal(st2.mean, 2.0 * st1.mean)
    assert st1.total_steps == st2.total_steps > 256 * 10_000 * 50
    # the tree kernel against the brute-force scan kernel, walk for walk, on a subset
    sub = sc.points[::4]
    tv, ts = s1.solve_walks(sub, nWalks=256, maxSteps=sc.max_steps, eps=sc.eps, seed=23)
    s1.set_segment_tree(-1)
    bv, bs = s1.solve_walks(sub, nWalks=256, maxSteps=sc.max_steps, eps=sc.eps, seed=23)
    assert s1.last_timing["tree"] == 0
    np.testing.assert_array_equal(ts, bs)
    np.testing.assert_array_equal(tv.view(np.uint32), bv.view(np.uint32))


def test_c5_wenner_survey_batches_equal_single_source_solves(gpu_available):
    from dcrmontecarlo_amd import survey

    sc = _c5(n_electrodes=40, n_walks=256)
    res = survey.run_wenner_survey(sc, 1e-2, n_walks=256, seed=3)
    Q = len(res.quadripoles)
    assert Q == 37 and res.launches == len(list(survey.wenner_batches(40, 1)))
    assert np.all(np.isfinite(res.model.dv)) and np.all(np.isfinite(res.background.dv))
    # quadripole q from a single-source solve of its own transmitter, same group seed
    sm = sc.solver(device=0)
    for g, (j0, j1, t0, t1) in enumerate(survey.wenner_batches(40, 1)):
        gseed = (3 * 0x9E3779B1 + g) & (2**64 - 1)
        for q in (t0, t1 - 1):
            if not (j0 <= q + 1 < j1 and j0 <= q + 2 < j1):
                continue
            sm.setSourceTerm(survey.dipole_source(sc.points[q], sc.points[q + 3], 0.5))
            u, st = sm.solve(sc.points[j0:j1], nWalks=256, maxSteps=sc.max_steps, eps=sc.eps, seed=gseed,
                             return_stats=True)
            assert st.mean[q + 1 - j0] - st.mean[q + 2 - j0] == res.model.dv[q]


def test_long_tree_with_wide_leaves_steps_down_its_staging(gpu_available):
    """25,000 segments in leaves of 32 keep the records under the 64-KB
    staging budget while the Neumann vertices (200 KB) cannot join them in LDS. The
    host must step down to records-only staging (not build a kernel that reads
    vertices it never staged); the tree kernel's walks equal the scan kernel's bit for
    bit."""
    sc = _c5(n_electrodes=32, n_walks=1, n_segments=25_000)
    s = sc.solver(device=0)
    s.set_segment_tree(0, 32)
    pts = sc.points[::4]
    tv, ts = s.solve_walks(pts, nWalks=128, maxSteps=sc.max_steps, eps=sc.eps, seed=41)
    assert s.last_timing["tree"] == 1
    s.set_segment_tree(-1)
    bv, bs = s.solve_walks(pts, nWalks=128, maxSteps=sc.max_steps, eps=sc.eps, seed=41)
    assert s.last_timing["tree"] == 0
    np.testing.assert_array_equal(ts, bs)
    np.testing.assert_array_equal(tv.view(np.uint32), bv.view(np.uint32))


def _with_options(s, opts):
    for key, val in opts.items():
        s.set_option(key, val)
    return s


@pytest.mark.parametrize("opts", [{"pool_slots": 1, "pool_near_waves": 0},
                                  {"pool_slots": 3, "pool_near_waves": 16, "pool_near": 1.0},
                                  {"pool_near_waves": 1, "pool_near": 0.01}, {}])
@pytest.mark.parametrize("physical", [False, True])
def test_c5_walk_pools_change_no_bits(gpu_available, opts, physical):
    """The tree kernels' walk pools (wost_walk.h) move whole walks between a workgroup's
    waves: every walk's value and step count equal those without pools, for tiny pools
    (one slot: constant parking pressure), near classes that take every walk, narrow
    near margins, and the defaults (wost_set_option)."""
    sc = _c5(physical=physical)
    pts = sc.points[::4][:64]
    s0 = _with_options(sc.solver(device=0), {"tree_pool": 0})
    v0, k0 = s0.solve_walks(pts, nWalks=1024, maxSteps=sc.max_steps, eps=sc.eps, seed=31)
    assert s0.last_timing["tree"] == 1
    s1 = _with_options(sc.solver(device=0), opts)
    v1, k1 = s1.solve_walks(pts, nWalks=1024, maxSteps=sc.max_steps, eps=sc.eps, seed=31)
    np.testing.assert_array_equal(np.asarray(k1), np.asarray(k0))
    np.testing.assert_array_equal(np.asarray(v1).view(np.uint32), np.asarray(v0).view(np.uint32))


def test_c5_walk_pools_change_no_bits_with_many_sources(gpu_available):
    """Multi-source walks (NS = 6: six totals travel with each parked walk) with one-slot
    pools equal the solve without pools, value for value and step for step."""
    from dcrmontecarlo_amd import survey

    sc = _c5(n_electrodes=64, n_walks=512)
    srcs = [survey.dipole_source(sc.points[q], sc.points[q + 3], 0.5) for q in range(0, 60, 10)]
    pts = sc.points[::2][:32]
    out = []
    for opts in ({"tree_pool": 0}, {"tree_pool": 1, "pool_slots": 1, "pool_near_waves": 0}):
        s = _with_options(sc.solver(device=0), opts)
        out.append(s.solve_sources_walks(pts, srcs, nWalks=512, maxSteps=sc.max_steps, eps=sc.eps, seed=9))
    (v0, k0), (v1, k1) = out
    assert v0.shape == (len(srcs), len(pts), 512)
    np.testing.assert_array_equal(k1, k0)
    np.testing.assert_array_equal(v1.view(np.uint32), v0.view(np.uint32))


def test_c5_walk_pools_change_no_bits_in_walk_range_solves(gpu_available):
    """Walk-range solves (wost_solve_range, the multi-GPU shard unit: a launch's local
    walks map to point ranges) with one-slot pools equal those without pools."""
    sc = _c5()
    pts = sc.points[::8][:24]
    out = []
    for opts in ({"tree_pool": 0}, {"tree_pool": 1, "pool_slots": 1, "pool_near_waves": 1}):
        s = _with_options(sc.solver(device=0), opts)
        out.append(s.solve_range(pts, 8192, 4096, 8192, sc.max_steps, sc.eps, 21))
    assert out[0].shape[0] == len(pts)
    np.testing.assert_array_equal(out[1], out[0])


@pytest.mark.parametrize("name", ["wenner_topography", "wenner_topography_physical"])
def test_c5_fused_bruteforce_scan_equals_separate_scans(gpu_available, name):
    """The brute-force scan kernel (set_segment_tree(-1)) runs both Neumann queries of a
    step in one pass with the per-vertex line filter (wost_device.h neumann_scan_both):
    walk for walk the bits of the two separate full scans (option fused_scan = 0, the
    round-4 kernel) and of the segment tree."""
    from dcrmontecarlo_amd import scenarios as S

    sc = S.ALL[name](n_electrodes=64, n_walks=1)
    pts = sc.points[::2]
    runs = {}
    for label in ("fused", "separate", "tree"):
        s = sc.solver(device=0)
        if label != "tree":
            s.set_segment_tree(-1)
        if label == "separate":
            s.set_option("fused_scan", 0)
        runs[label] = s.solve_walks(pts, nWalks=512, maxSteps=sc.max_steps, eps=sc.eps, seed=29)
        assert s.last_timing["tree"] == (1 if label == "tree" else 0)
    for label in ("separate", "tree"):
        np.testing.assert_array_equal(runs["fused"][1], runs[label][1], err_msg=label)
        np.testing.assert_array_equal(runs["fused"][0].view(np.uint32), runs[label][0].view(np.uint32), err_msg=label)


def test_fused_bruteforce_scan_from_global_memory(gpu_available):
    """A Neumann polyline too long to stage in LDS even with one 1024-thread workgroup per
    CU (20,000 segments: 160 KB of vertices) is scanned from global memory through the
    scalar unit (neumann_scan_both<SCALAR>): walk for walk the segment tree's bits."""
    from dcrmontecarlo_amd import scenarios as S

    sc = S.wenner_topography(n_electrodes=32, n_walks=1, n_segments=20_000)
    pts = sc.points[::2]
    runs = {}
    for label in ("scan", "tree"):
        s = sc.solver(device=0)
        if label == "scan":
            s.set_segment_tree(-1)
        runs[label] = s.solve_walks(pts, nWalks=128, maxSteps=sc.max_steps, eps=sc.eps, seed=31)
        assert s.last_timing["tree"] == (1 if label == "tree" else 0)
    np.testing.assert_array_equal(runs["scan"][1], runs["tree"][1])
    np.testing.assert_array_equal(runs["scan"][0].view(np.uint32), runs["tree"][0].view(np.uint32))
