"""C5 (the 10k-segment topography with the notebook's fields) pinned to the
reference itself, on CPU: tools/gen_fixtures.py ran the reference's own code on it
(--only c5_fields,c5_kats and the wenner_topography replay) and committed

* fields_wenner_topography[_physical].npz: g, f, alpha, sigma' at 256 points (half of
  them within 4 units of the surface) and the reference's sigma_bar (bounding box
  solvers/WoStSolver.py:37-43, gridSampleMinMax utils.py:65-120, fallback :130-136);
* geometry_kats_c5.npz: the five PolyLinesSimple queries (geometry/PolylinesSimple.py:
  25-197) at 320 positions of recorded C5 walks, 240 of them within 4 units of the
  surface;
* replay_wenner_topography.npz: _solveUnified (:162-316) on libwost's Philox stream,
  8 electrodes x 32 walks, 57,613 steps.

The oracle (oracle/wost_oracle.c) must reproduce them with its OWN sigma_bar, and the
segment tree (the device code, built for the host) must return the reference's
queries. Tolerances: the reference's torch kernels on 10k-element tensors round a few
results differently from its scalar arithmetic (1-ulp differences in distance and in
the hit point; silhouette distances, silhouette masks, hit flags and normals are
bit-identical), so those are compared within 2 ulps of the coordinates; every step
of a walk feeds such ulps back in, so the replayed walks are compared against the
oracle's own 1-ulp chaos measured on the same walks."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from conftest import golden
from oracle import oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
K = "topo10k_walk__"


def ulps(a, b, scale=None):
    """|a - b| in units of the float32 spacing at max(|a|, |b|, scale) (NaN/inf equal: 0)."""
    a, b = np.asarray(a, np.float32), np.asarray(b, np.float32)
    same = (a == b) | (np.isnan(a) & np.isnan(b))
    m = np.maximum(np.abs(a), np.abs(b))
    if scale is not None:
        m = np.maximum(m, np.asarray(scale, np.float32))
    sp = np.spacing(m.astype(np.float32))
    return np.where(same, 0.0, np.abs(a.astype(np.float64) - b) / sp)


def check_against_reference_kats(sil, hit, z, what):
    """silhouette distance bit for bit; intersectPolylines: found and normal bit for bit,
    the hit point within 2 ulps of the query's largest coordinate (x + t d rounds at
    that scale)."""
    rs, ri = z[K + "silhouette_distance"], z[K + "intersect"]
    np.testing.assert_array_equal(sil.view(np.uint32), rs.view(np.uint32), err_msg=f"{what}: silhouetteDistance")
    np.testing.assert_array_equal(hit[:, 2:5].view(np.uint32), ri[:, 2:5].view(np.uint32),
                                  err_msg=f"{what}: intersectPolylines normal / found")
    P = z[K + "points"]
    scale = np.maximum(np.abs(P).max(1), np.abs(ri[:, 0:2]).max(1))[:, None]
    u = ulps(hit[:, 0:2], ri[:, 0:2], scale)
    assert u.max() <= 2.0, (what, u.max())
    assert np.isfinite(rs).sum() > 200 and ri[:, 4].sum() > 100     # both queries exercised


@pytest.fixture(scope="module")
def kats():
    return golden("geometry_kats_c5.npz")


def test_oracle_scans_reproduce_reference_c5_kats(kats):
    z = kats
    V, P, D, R = (z[K + k] for k in ("verts", "points", "dirs", "radii"))
    sil = O.geometry("silhouetteDistance", V, P)
    hit = O.geometry("intersectPolylines", V, P, D, R)
    check_against_reference_kats(sil, hit, z, "oracle")
    np.testing.assert_array_equal(O.geometry("isSilhouette", V, P), z[K + "is_silhouette"])
    assert ulps(O.geometry("distance", V, P), z[K + "distance"]).max() <= 2.0


@pytest.fixture(scope="module")
def tree_lib(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("c5tree") / "libtree_check.so")
    src = [os.path.join(HERE, "native", "tree_check.cpp"), os.path.join(REPO, "dcrmontecarlo_amd", "csrc", "wost_tree.cpp")]
    subprocess.run(["/opt/rocm/bin/hipcc", "-O2", "-std=c++17", "-fPIC", "-shared", "--offload-arch=gfx950",
                    "-I" + os.path.join(REPO, "include"), "-x", "hip", src[0], "-x", "c++", src[1], "-o", out],
                   check=True)
    lib = ctypes.CDLL(out)
    fp = ctypes.POINTER(ctypes.c_float)
    lib.tree_query.argtypes = [fp, ctypes.c_int, ctypes.c_int, fp, fp, fp, ctypes.c_long, fp, fp]
    lib.tree_query.restype = ctypes.c_int
    return lib


@pytest.mark.parametrize("leaf", [10, 1, 32])
def test_host_tree_reproduces_reference_c5_kats(kats, tree_lib, leaf):
    """The segment tree's traversal (wost_device.h, the kernels' code built for the host)
    at the reference's query points: the reference's answers, and the oracle scan's bits."""
    z = kats
    V, P, D, R = (np.ascontiguousarray(z[K + k], np.float32) for k in ("verts", "points", "dirs", "radii"))
    n = P.shape[0]
    sil, hit = np.empty(n, np.float32), np.empty((n, 5), np.float32)
    f = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))
    assert tree_lib.tree_query(f(V), V.shape[0], leaf, f(P), f(D), f(R), n, f(sil), f(hit)) == 0
    check_against_reference_kats(sil, hit, z, f"host tree (leaf {leaf})")
    np.testing.assert_array_equal(sil.view(np.uint32), O.geometry("silhouetteDistance", V, P).view(np.uint32))
    np.testing.assert_array_equal(hit.view(np.uint32), O.geometry("intersectPolylines", V, P, D, R).view(np.uint32))


@pytest.mark.parametrize("name", ["wenner_topography", "wenner_topography_physical"])
def test_oracle_fields_and_sigma_bar_c5(name):
    """The C5 field restatements against the reference's callables, and the oracle's own
    sigma_bar and sigma' against the reference's (rel 1e-6: the same grid and fallback)."""
    from dcrmontecarlo_amd import scenarios as S

    z = golden(f"fields_{name}.npz")
    sc = S.ALL[name]()
    np.testing.assert_array_equal(sc.neumann, z["neumann"])
    np.testing.assert_array_equal(sc.dirichlet, z["dirichlet"])
    P = z["points"]
    for key in ("f", "alpha"):
        ref = z[key]
        scale = max(np.abs(ref).max(), 1e-30)
        np.testing.assert_allclose(O.field_value(getattr(sc, key), P), ref, rtol=1e-5, atol=1e-6 * scale, err_msg=key)
    pb = O.Problem(z["dirichlet"], z["neumann"], sc.g, sc.f, sc.sigma, sc.alpha)
    assert pb.sigma_bar() == pytest.approx(float(z["sigma_bar"]), rel=1e-6)
    sp = pb.sigma_prime(P).astype(np.float64)
    ref = z["sigma_prime"]
    fin = np.isfinite(ref)
    assert fin.sum() > 200
    np.testing.assert_allclose(sp[fin], ref[fin], rtol=2e-3, atol=1e-5 * np.abs(ref[fin]).max())


def c5_replay_agreement(v, s, z):
    """(share of walks with the reference's step count and value within 1e-3, share of
    walk values within 1e-4) of per-walk results v, s against the replay fixture."""
    rv, rs = z["walk_values"], z["walk_steps"]
    scale = max(float(np.abs(rv).max()), 1e-30)
    same = (np.asarray(s) == rs) & (np.abs(v - rv) <= 1e-3 * np.abs(rv) + 1e-5 * scale)
    close = np.abs(v - rv) <= 1e-4 * np.abs(rv) + 1e-6 * scale
    return float(same.mean()), float(close.mean())


def test_oracle_replays_reference_c5_walks():
    """The reference's C5 walks on the Philox stream, with the oracle's OWN sigma_bar: the
    share of identical walks must reach the oracle's agreement with itself under a 1-ulp
    change of the step direction on the same walks (measured here; ~0.81), and the
    per-electrode means agree within 1e-3 relative."""
    from dcrmontecarlo_amd import scenarios as S

    z = golden("replay_wenner_topography.npz")
    sc = S.wenner_topography(n_walks=1)
    pb0 = O.Problem(z["dirichlet"], z["neumann"], sc.g, sc.f, sc.sigma, sc.alpha)
    sb = pb0.sigma_bar()
    assert sb == pytest.approx(float(z["sigma_bar"]), rel=1e-6)
    pb = O.Problem(z["dirichlet"], z["neumann"], sc.g, sc.f, sc.sigma, sc.alpha, sigma_bar=sb)
    args = (z["points"], int(z["n_walks"]), int(z["max_steps"]), float(z["eps"]), int(z["seed"]))
    v, s = pb.solve_walks(*args)
    try:
        O.set_direction_perturbation(1.2e-7)
        pv, ps = pb.solve_walks(*args)
    finally:
        O.set_direction_perturbation(0.0)
    scale = max(float(np.abs(v).max()), 1e-30)
    chaos = float(((ps == s) & (np.abs(pv - v) <= 1e-3 * np.abs(v) + 1e-5 * scale)).mean())
    same, close = c5_replay_agreement(v, s, z)
    assert chaos > 0.6 and same >= chaos, (same, chaos)
    assert close >= 0.95, close
    n = len(z["points"])
    m_o = v.astype(np.float64).reshape(n, -1).mean(1)
    m_r = z["walk_values"].reshape(n, -1).mean(1)
    np.testing.assert_allclose(m_o, m_r, rtol=1e-3, atol=1e-6 * np.abs(m_r).max())


# ---------------------------------------------------------------- C5 apparent resistivity (G13)
def oracle_wenner_walks(ref, sc):
    """survey.wenner_replay_walks' solver on the oracle: only the receivers' walk ranges."""
    from dcrmontecarlo_amd import fields as F

    def solve_walks(f, pts, srcs, W, seed, rows):
        vals = np.zeros((len(srcs), len(pts), W), np.float32)
        steps = np.zeros((len(pts), W), np.uint32)
        alpha = sc.alpha if f == 0 else F.const(ref.alpha_bg)
        for j, src in enumerate(srcs):
            pb = O.Problem(sc.dirichlet, sc.neumann, sc.g, src, sc.sigma, alpha, sigma_bar=ref.sigma_bar)
            for e in rows:
                v, st = pb.solve_walks(pts, W, sc.max_steps, sc.eps, seed, wid_begin=e * W, wid_end=(e + 1) * W)
                vals[j, e], steps[e] = v, st
        return vals, steps

    return solve_walks


# the oracle's share of the reference's C5 Wenner walks it reproduces on the whole fixture
# (32 quadripoles x both receivers x 64 walks x model + background), measured with
# survey.compare_wenner_replay over oracle_wenner_walks (round 6; ~6 min of CPU for the
# literal survey's 204-step walks, so the CPU test below checks 4 of the quadripoles):
# the device's floor in tests/test_gpu_c5_reference.py
ORACLE_RHO_IDENTICAL = {"wenner_topography": 0.918, "wenner_topography_physical": 0.982}


@pytest.mark.parametrize("name", ["wenner_topography", "wenner_topography_physical"])
def test_c5_rho_replay_fixture_is_the_survey_layout(name):
    """G13 (rho_replay_<name>.npz: the physical survey, and since round 6 the literal one
    the bench times): the receivers are the quadripoles' M and N, their groups and seeds
    those of survey.run_wenner_survey, model and background walks share their paths
    (common random numbers), 32 quadripoles."""
    from dcrmontecarlo_amd import scenarios as S
    from dcrmontecarlo_amd import survey as SV

    z = golden(f"rho_replay_{name}.npz")
    ref = SV.load_wenner_replay(os.path.join(HERE, "golden", f"rho_replay_{name}.npz"))
    assert ref.source == f"rho_replay_{name}.npz" and len(ref.quadripoles) == 32
    sc = S.ALL[name](n_walks=1)
    np.testing.assert_array_equal(ref.points, sc.points)
    np.testing.assert_array_equal(ref.receivers, ref.quadripoles[:, 1:3])
    batches = list(SV.wenner_batches(len(sc.points)))
    for i in range(len(ref.quadripoles)):
        for k in range(2):
            g = int(ref.groups[i, k])
            j0, j1, t0, t1 = batches[g]
            assert j0 <= ref.receivers[i, k] < j1 and t0 <= ref.quadripoles[i, 0] < t1
            assert int(z["group_seeds"][i, k]) == SV.group_seed(ref.survey_seed, g)
    assert bool(z["common_paths"]) and np.array_equal(ref.model_steps, ref.background_steps)
    assert ref.sigma_bar == pytest.approx(float(golden(f"fields_{name}.npz")["sigma_bar"]), rel=1e-12)


@pytest.mark.parametrize("name", ["wenner_topography", "wenner_topography_physical"])
def test_oracle_replays_reference_c5_rho_a(name):
    """The oracle on the reference's C5 Wenner walks (4 of the 32 quadripoles): the walks
    identical as often as on the whole fixture (ORACLE_RHO_IDENTICAL) less 0.03, and every
    quadripole's dV and rho_a within the bound the diverged walks allow
    (survey.compare_wenner_replay)."""
    from dcrmontecarlo_amd import scenarios as S
    from dcrmontecarlo_amd import survey as SV

    ref = SV.load_wenner_replay(os.path.join(HERE, "golden", f"rho_replay_{name}.npz"))
    ref = SV.wenner_replay_subset(ref, [3, 12, 19, 28])
    sc = S.ALL[name](n_walks=1)
    out = SV.compare_wenner_replay(*SV.wenner_replay_walks(ref, oracle_wenner_walks(ref, sc)), ref)
    assert out["walks_identical"] >= ORACLE_RHO_IDENTICAL[name] - 0.03, out["walks_identical"]
    assert out["all_within_tolerance"], out
