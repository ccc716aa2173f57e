"""The Neumann segment tree returns the same bits as the full scans it replaces.

CPU: the device geometry (wost_device.h, __host__ __device__) is compiled for
the host together with the tree builder, and fuzzed against the scans of
geometry/PolylinesSimple.py (silhouetteDistance :83-102 in its use
min(dn, dD) of solvers/WoStSolver.py:211-212, and intersectPolylines
:134-197) on random, near-boundary and collinear/near-parallel queries.
GPU: whole walks with the tree kernels vs the scan kernels, walk for walk.
"""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from dcrmontecarlo_amd import scenarios as S

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("tree") / "libtree_check.so")
    src = [os.path.join(HERE, "native", "tree_check.cpp"), os.path.join(REPO, "dcrmontecarlo_amd", "csrc", "wost_tree.cpp")]
    # the geometry is __host__ __device__ HIP: compile it as HIP, call it on the host
    subprocess.run(["/opt/rocm/bin/hipcc", "-O2", "-std=c++17", "-fPIC", "-shared", "--offload-arch=gfx950",
                    "-I" + os.path.join(REPO, "include"), "-x", "hip", src[0], "-x", "c++", src[1], "-o", out],
                   check=True)
    lib = ctypes.CDLL(out)
    fp = ctypes.POINTER(ctypes.c_float)
    lib.tree_check.argtypes = [fp, ctypes.c_int, ctypes.c_int, fp, fp, fp, fp, ctypes.c_long,
                               ctypes.POINTER(ctypes.c_long)]
    lib.tree_check.restype = ctypes.c_int
    lib.tree_check_nearest.argtypes = [fp, ctypes.c_int, ctypes.c_int, fp, fp, fp, ctypes.c_long,
                                       ctypes.POINTER(ctypes.c_long)]
    lib.tree_check_nearest.restype = ctypes.c_int
    lib.tree_check_stop.argtypes = [fp, ctypes.c_int, ctypes.c_int, fp, fp, ctypes.c_float, ctypes.c_float,
                                    ctypes.c_long, ctypes.POINTER(ctypes.c_long)]
    lib.tree_check_stop.restype = ctypes.c_int
    lib.tree_build_depth.argtypes = [fp, ctypes.c_int, ctypes.c_int]
    lib.tree_build_depth.restype = ctypes.c_int
    return lib


def stop2_of(rmin):
    """The largest float32 whose (correctly rounded) sqrt is <= rmin (wost_api.hip silhouette_stop2)."""
    rmin = np.float32(rmin)
    x = np.float32(rmin * rmin)
    while x > 0 and np.sqrt(x) > rmin:
        x = np.nextafter(x, np.float32(0))
    while np.sqrt(np.nextafter(x, np.float32(np.inf))) <= rmin:
        x = np.nextafter(x, np.float32(np.inf))
    return x


def run(lib, verts, pts, dirs, radii, dd, leaf=8):
    f = lambda a: np.ascontiguousarray(a, np.float32)
    verts, pts, dirs, radii, dd = f(verts), f(pts), f(dirs), f(radii), f(dd)
    out = (ctypes.c_long * 4)()
    p = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))
    rc = lib.tree_check(p(verts), verts.shape[0], leaf, p(pts), p(dirs), p(radii), p(dd), pts.shape[0], out)
    assert rc == 0
    return list(out)


def queries(rng, verts, n):
    """Mix of domain points, points near the polyline, and rays from the line of
    a segment along (almost) its direction."""
    lo, hi = verts.min(0), verts.max(0)
    span = hi - lo + 1.0
    k = n // 3
    a = lo - 0.2 * span + rng.random((k, 2)) * 1.4 * span                       # anywhere
    i = rng.integers(0, len(verts) - 1, n - k)
    t = rng.random(n - k)
    base = verts[i] + t[:, None] * (verts[i + 1] - verts[i])
    off = rng.normal(size=(n - k, 2)) * 10.0 ** rng.uniform(-6, 1, (n - k, 1))   # near the polyline
    b = base + off
    pts = np.concatenate([a, b]).astype(np.float32)
    th = rng.random(n) * 2 * np.pi
    dirs = np.stack([np.cos(th), np.sin(th)], 1)
    # a third of the near points shoot along their segment (collinear / near-parallel)
    m = n - k
    sel = k + np.arange(m // 2)
    u = verts[i[: m // 2] + 1] - verts[i[: m // 2]]
    rot = rng.normal(size=m // 2) * 10.0 ** rng.uniform(-9, -2, m // 2)
    c, s = np.cos(rot), np.sin(rot)
    dirs[sel] = np.stack([u[:, 0] * c - u[:, 1] * s, u[:, 0] * s + u[:, 1] * c], 1) * rng.choice([-1, 1], (m // 2, 1))
    radii = 10.0 ** rng.uniform(-2, 3, n)
    dd = 10.0 ** rng.uniform(-1, 3.5, n)
    dd[rng.random(n) < 0.1] = np.inf
    return pts, dirs.astype(np.float32), radii, dd


@pytest.mark.parametrize("leaf", [1, 3, 8, 32])
def test_tree_matches_scan_topography(harness, leaf):
    rng = np.random.default_rng(leaf)
    verts = S.topography(2000)
    counts = run(harness, verts, *queries(rng, verts, 60000), leaf=leaf)
    assert counts[0] == 0 and counts[1] == 0, counts
    assert counts[2] > 1000 and counts[3] > 1000, counts     # both queries exercised


def test_tree_matches_scan_full_topography(harness):
    rng = np.random.default_rng(7)
    verts = S.topography(10_000)
    counts = run(harness, verts, *queries(rng, verts, 60000))
    assert counts[0] == 0 and counts[1] == 0, counts


@pytest.mark.parametrize("rmin", [0.45, 0.05, 2.0])
def test_tree_early_stop_keeps_the_step_radius(harness, rmin):
    """silhouette_distance_tree stops once a silhouette vertex lies within rmin: the
    step radius max(rmin, min(dn, dd)) is then rmin whatever the rest of the polyline
    holds. Checked against the full scan on near-surface points of the C5 topography."""
    rng = np.random.default_rng(int(rmin * 100))
    verts = S.topography(10_000)
    pts, _, _, dd = queries(rng, verts, 40000)
    stop2 = stop2_of(rmin)
    assert np.sqrt(stop2) <= np.float32(rmin) < np.sqrt(np.nextafter(stop2, np.float32(np.inf)))
    f = lambda a: np.ascontiguousarray(a, np.float32)
    p = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))
    out = (ctypes.c_long * 3)()
    verts, pts, dd = f(verts), f(pts), f(dd)
    assert harness.tree_check_stop(p(verts), verts.shape[0], 8, p(pts), p(dd), float(rmin), float(stop2),
                                   pts.shape[0], out) == 0
    assert out[0] == 0, list(out)
    assert out[1] > 100, list(out)        # the early stop was exercised


def test_tree_matches_scan_at_c5_walk_positions(harness):
    """The positions C5 walks actually visit (30,000 steps recorded on the device by
    tools/c5_paths.py: electrodes 0.1 below the surface, near-surface steps, walkers
    escaped to |y| ~ 1e6), each with its Dirichlet distance, random directions and
    the step radius: the tree's queries equal the full scans bit for bit."""
    z = np.load(os.path.join(HERE, "golden", "c5_walk_positions.npz"))
    rng = np.random.default_rng(11)
    n = len(z["points"])
    th = rng.random(n) * 2 * np.pi
    dirs = np.stack([np.cos(th), np.sin(th)], 1)
    radii = np.minimum(z["dd"], 10.0 ** rng.uniform(-1, 3, n))
    for leaf in (8, 10, 16):
        counts = run(harness, S.topography(10_000), z["points"], dirs, radii, z["dd"], leaf=leaf)
        assert counts[0] == 0 and counts[1] == 0, (leaf, counts)
        assert counts[2] > 100 and counts[3] > 1000, counts


SHAPES = ["circle", "zigzag", "random_walk", "degenerate", "far_offset"]


@pytest.mark.parametrize("shape", SHAPES)
def test_tree_matches_scan_shapes(harness, shape):
    rng = np.random.default_rng(SHAPES.index(shape))
    if shape == "circle":                                   # closed, every vertex a silhouette candidate
        th = np.linspace(0, 2 * np.pi, 513)
        verts = np.stack([40 * np.cos(th), 40 * np.sin(th)], 1)
    elif shape == "zigzag":                                 # direction cones too wide to prune
        x = np.linspace(-50, 50, 801)
        verts = np.stack([x, np.where(np.arange(801) % 2, 1.0, -1.0)], 1)
    elif shape == "random_walk":
        verts = np.cumsum(rng.normal(size=(1500, 2)), 0)
    elif shape == "degenerate":                             # repeated vertices, zero-length segments
        x = np.repeat(np.linspace(-10, 10, 300), 2)
        verts = np.stack([x, np.sin(x)], 1)
    else:                                                   # large coordinates: the tolerances scale
        verts = S.topography(3000).astype(np.float64) + np.array([3.0e4, -2.0e4])
    verts = verts.astype(np.float32)
    counts = run(harness, verts, *queries(rng, verts, 40000))
    assert counts[0] == 0 and counts[1] == 0, counts


def test_tree_small_polylines(harness):
    rng = np.random.default_rng(3)
    for nv in (2, 3, 4, 9, 17):
        verts = rng.normal(size=(nv, 2)).astype(np.float32) * 5
        counts = run(harness, verts, *queries(rng, verts, 5000))
        assert counts[0] == 0 and counts[1] == 0, (nv, counts)


@pytest.mark.gpu
def test_gpu_tree_walks_match_scan_walks(gpu_available):
    """C5-shaped problem (2000-segment topography, reduced): every walk of the tree
    kernel equals the scan kernel's walk, value and step count, for both the
    field-specialised and the precompiled kernels."""
    sc = S.wenner_topography(n_electrodes=16, n_walks=512, n_segments=2000)
    res = {}
    for tree in (False, True):
        for jit in (True, False):
            s = sc.solver(device=0)
            s.set_segment_tree(0 if tree else -1)
            s.set_jit(jit)
            v, st = s.solve_walks(sc.points, nWalks=sc.n_walks, maxSteps=sc.max_steps, eps=sc.eps, seed=9)
            assert s.last_timing["tree"] == int(tree)
            res[(tree, jit)] = (v.ravel(), st.ravel())
    ref = res[(False, True)]
    for key, (v, st) in res.items():
        np.testing.assert_array_equal(st, ref[1], err_msg=str(key))
        np.testing.assert_array_equal(v.view(np.uint32), ref[0].view(np.uint32), err_msg=str(key))


@pytest.mark.gpu
@pytest.mark.parametrize("knobs", [
    {"leaf": 1}, {"leaf": 32},
    {"tree_share": 0}, {"tree_share": 64, "tree_share_min": 1},
    {"tree_share_descent": 0, "tree_batch": 1},
    {"tree_batch": 2, "jit_waves": 6}, {"tree_lds": 0}, {"tree_lds": 1},
    {"tree_lds": 0, "tree_share": 0}])
def test_gpu_cooperative_tree_variants_match_scan_walks(gpu_available, knobs):
    """The wave-cooperative tree queries (wost_walk.h: hand-outs of pending subtrees,
    batched record loads, records staged in LDS or read through L1/L2) under every
    hand-out threshold, leaf size and load batch (wost_set_segment_tree, wost_set_option)
    give the scan kernel's walks bit for bit (the answers are order-independent
    minima; only the visiting order and the lanes doing the visits change)."""
    sc = S.wenner_topography(n_electrodes=16, n_walks=512, n_segments=2000)
    s = sc.solver(device=0)
    s.set_segment_tree(-1)
    v0, st0 = s.solve_walks(sc.points, nWalks=sc.n_walks, maxSteps=sc.max_steps, eps=sc.eps, seed=21)
    s = sc.solver(device=0)
    for k, v in knobs.items():
        if k == "leaf":
            s.set_segment_tree(64, v)
        else:
            s.set_option(k, v)
    v1, st1 = s.solve_walks(sc.points, nWalks=sc.n_walks, maxSteps=sc.max_steps, eps=sc.eps, seed=21)
    assert s.last_timing["tree"] == 1 and s.last_timing["jit"]
    np.testing.assert_array_equal(st1, st0)
    np.testing.assert_array_equal(v1.view(np.uint32), v0.view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("n_segments,staged", [(10_000, True), (40_000, False)])
def test_gpu_tree_lds_staging_levels(gpu_available, n_segments, staged):
    """The field-specialised tree kernels stage the tree's records and the Neumann
    vertices in LDS (one 1024-thread workgroup per CU) when they fit -- C5's 10k
    segments do -- and step down to reading them through L1/L2 from 256-thread
    workgroups when they do not (40k segments: 175 KB of records); either way the
    walks are the scan kernel's, bit for bit."""
    sc = S.wenner_topography(n_electrodes=8, n_walks=128, n_segments=n_segments)
    res = []
    for tree in (False, True):
        s = sc.solver(device=0)
        s.set_segment_tree(0 if tree else -1)
        v, st = s.solve_walks(sc.points, nWalks=sc.n_walks, maxSteps=sc.max_steps, eps=sc.eps, seed=5)
        assert s.last_timing["tree"] == int(tree)
        res.append((v.ravel(), st.ravel(), s.last_timing["grid_blocks"]))
    np.testing.assert_array_equal(res[1][1], res[0][1])
    np.testing.assert_array_equal(res[1][0].view(np.uint32), res[0][0].view(np.uint32))
    # 1,024 walks: one 1024-thread workgroup when staged, four 256-thread ones otherwise
    assert res[1][2] == (1 if staged else 4), res[1][2]


def run_nearest(lib, verts, pts, dirs, radii, leaf=8):
    f = lambda a: np.ascontiguousarray(a, np.float32)
    verts, pts, dirs, radii = f(verts), f(pts), f(dirs), f(radii)
    out = (ctypes.c_long * 2)()
    p = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))
    assert lib.tree_check_nearest(p(verts), verts.shape[0], leaf, p(pts), p(dirs), p(radii), pts.shape[0], out) == 0
    return list(out)


@pytest.mark.parametrize("leaf", [1, 8, 32])
def test_tree_nearest_crossing_matches_scan(harness, leaf):
    """compat="fixed" (Q1 corrected): the nearest crossing along the ray through the
    tree equals intersect_polylines_ray's full scan bit for bit -- the hit point and
    the segment whose normal the walk turns on -- on the 10k-segment topography and
    a closed zig-zag (ties at shared vertices keep the lower segment index)."""
    rng = np.random.default_rng(77 + leaf)
    topo = S.topography(10_000)
    pts, dirs, radii, _ = queries(rng, topo.astype(np.float64), 60_000)
    bad, hits = run_nearest(harness, topo, pts, dirs, radii, leaf)
    assert bad == 0 and hits > 1000
    ang = np.linspace(0, 2 * np.pi, 401)
    zig = np.stack([np.cos(ang) * (1 + 0.3 * (np.arange(401) % 2)), np.sin(ang) * (1 + 0.3 * (np.arange(401) % 2))], 1)
    zig[-1] = zig[0]
    pts, dirs, radii, _ = queries(rng, zig, 60_000)
    # rays aimed exactly at vertices: the crossing is shared by two segments
    k = 5000
    j = rng.integers(1, 400, k)
    pts[:k] = (zig[j] * 0.3).astype(np.float32)
    dirs[:k] = (zig[j] - pts[:k]).astype(np.float32)
    bad, hits = run_nearest(harness, zig.astype(np.float32), pts, dirs, radii, leaf)
    assert bad == 0 and hits > 1000


def test_tree_depth_limit(harness):
    """The traversals keep 4 pending-child bits per level in 32 bits (wost_tree.h
    kTreeMaxDepth = 8): the builder refuses a deeper tree, and libwost then retries with
    32-segment leaves (wost_api.hip ensure_tree) before failing loudly."""
    n = 65536 + 2   # 65537 segments: 4^8 one-segment leaves are one too few
    x = np.linspace(-1.0, 1.0, n, dtype=np.float32)
    xy = np.ascontiguousarray(np.stack([x, np.sin(x)], 1), np.float32)
    p = xy.ctypes.data_as(ctypes.POINTER(ctypes.c_float))
    assert harness.tree_build_depth(p, n - 1, 1) == 8     # 65535 segments
    assert harness.tree_build_depth(p, n, 1) == -1        # 65537 segments
    assert harness.tree_build_depth(p, n, 32) == 6
