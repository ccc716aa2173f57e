"""The walk kernels' work queue and launch shape (wost_walk.h refill, wost_api.hip
solve_impl): a walk's result depends only on its id, so every queue shape gives the
same bits.

Round 6: the launch shape is a function of the call alone (never of an earlier solve on
the handle): walks without a Neumann boundary start with static 64-walk chunks and a
grid of ~4 walks per lane; the host's dequeue size holds until a wave has finished walks,
after which each wave sizes its dequeues from its own measured mean steps and walk rate
(WalkArgs::adaptive). So a fresh handle's first solve -- the reference's only usage,
tests/testWostWithSource.py:110 -- runs the shape a warm handle runs, and each forced
shape (wost_set_option chunk0 / chunk_min / chunk_max / adaptive_chunk /
grid_blocks_per_cu) gives the default's walks bit for bit. The launch statistics
(wost_timing max_walk_steps, span/tail, the last wave) are checked against the walks.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SHAPE = ("grid_blocks", "blocks_per_cu", "block_threads", "chunk0", "chunk", "adaptive")



def _set_options(s) -> dict:
    """The handle's non-default options besides jit_race, which tests/conftest.py sets to 0
    on every GPU test's solver (its kernel compiled before its first solve)."""
    return {k: v for k, v in s.options_report()["non_default"].items() if k != "jit_race"}

def _walks(s, pts, W, sc, seed):
    v, st = s.solve_walks(pts, nWalks=W, maxSteps=sc.max_steps, eps=sc.eps, seed=seed)
    return np.asarray(v).view(np.uint32).copy(), np.asarray(st).copy()


def _scenario(name):
    from dcrmontecarlo_amd import scenarios as S

    kw = {"n_walks": 1} if name in ("dcr_dipole", "wenner_topography") else {}
    if name == "wenner_topography":
        kw["n_electrodes"] = 64
    return S.ALL[name](**kw)


@pytest.mark.parametrize("name, big, small", [
    ("poisson_square", (64, 4000), (3, 100)),       # short walks: static chunks, fewer workgroups
    ("poisson_square", (64, 4000), (64, 3000)),     # ... with dynamic chunks after the static ones
    ("dcr_dipole", (48, 2000), (5, 300)),           # long walks with a Neumann boundary
    ("wenner_topography", (64, 256), (8, 200)),     # the segment-tree kernel (no static chunks)
])
def test_launch_shape_is_a_function_of_the_call(gpu_available, name, big, small):
    """A fresh handle and a handle that just solved a different problem size launch the
    same shape for the same call, and their walks are identical."""
    sc = _scenario(name)
    pts_big = np.resize(sc.points, (big[0], 2)).astype(np.float32)
    pts_small = np.ascontiguousarray(pts_big[:small[0]])
    fresh = sc.solver(device=0)
    ref = _walks(fresh, pts_small, small[1], sc, seed=7)      # no previous solve
    shape = {k: fresh.last_timing[k] for k in SHAPE}
    warm = sc.solver(device=0)
    _walks(warm, pts_big, big[1], sc, seed=3)                 # another call first
    got = _walks(warm, pts_small, small[1], sc, seed=7)
    assert {k: warm.last_timing[k] for k in SHAPE} == shape
    again = _walks(warm, pts_small, small[1], sc, seed=7)     # the queue head reset by the reduce
    for g in (got, again):
        np.testing.assert_array_equal(g[1], ref[1])
        np.testing.assert_array_equal(g[0], ref[0])
    assert ref[1].sum() > 0
    assert shape["adaptive"] == (0 if name == "wenner_topography" else 1)   # tree kernels: host-sized dequeues


@pytest.mark.parametrize("name", ["poisson_square", "dcr_dipole", "wenner_topography"])
@pytest.mark.parametrize("opts", [{"adaptive_chunk": 0}, {"chunk0": 0}, {"chunk0": 1, "chunk_min": 1, "chunk_max": 1},
                                  {"chunk0": 1024, "chunk_max": 1024}, {"grid_blocks_per_cu": 1}])
def test_forced_queue_shapes_change_no_bits(gpu_available, name, opts):
    sc = _scenario(name)
    pts = np.ascontiguousarray(np.resize(sc.points, (16, 2)).astype(np.float32))
    ref = _walks(sc.solver(device=0), pts, 700, sc, seed=5)
    s = sc.solver(device=0)
    for k, v in opts.items():
        s.set_option(k, v)
    got = _walks(s, pts, 700, sc, seed=5)
    np.testing.assert_array_equal(got[1], ref[1])
    np.testing.assert_array_equal(got[0], ref[0])
    assert _set_options(s) == {k: float(v) for k, v in opts.items()}
    if "chunk_min" in opts or "adaptive_chunk" in opts:
        assert s.last_timing["adaptive"] == 0


def test_static_chunks_cover_every_walk(gpu_available):
    """Fewer walks than one static chunk per wave (the queue is never dequeued): every walk
    runs once, with the step counts of a handle that solved a larger problem first."""
    from dcrmontecarlo_amd import scenarios as S

    sc = S.ALL["laplace_square"]()
    pts = np.ascontiguousarray(sc.points[:2], np.float32)
    warm = sc.solver(device=0)
    _walks(warm, np.resize(sc.points, (64, 2)).astype(np.float32), 2000, sc, seed=1)
    for W in (1, 7, 64, 65):
        ref = _walks(sc.solver(device=0), pts, W, sc, seed=11)
        got = _walks(warm, pts, W, sc, seed=11)
        np.testing.assert_array_equal(got[1], ref[1])
        np.testing.assert_array_equal(got[0], ref[0])
        assert (got[1] > 0).all()


@pytest.mark.parametrize("name", ["poisson_square", "dcr_dipole"])
def test_launch_statistics(gpu_available, name):
    """wost_timing's launch statistics: the longest walk equals the walks' maximum; the
    busiest wave iterated at least that often; the tail follows the last dequeue and lies
    inside the launch's span, which the walk kernel's HIP-event time bounds."""
    sc = _scenario(name)
    s = sc.solver(device=0)
    pts = np.ascontiguousarray(np.resize(sc.points, (32, 2)).astype(np.float32))
    v, st = s.solve_walks(pts, nWalks=5000, maxSteps=sc.max_steps, eps=sc.eps, seed=2)
    t = s.last_timing
    assert t["max_walk_steps"] == int(np.max(st))
    assert t["max_wave_iters"] >= t["max_walk_steps"]
    assert t["last_wave_iters"] >= 1 and t["last_wave_ms"] > 0.0
    assert 0.0 <= t["tail_ms"] <= t["span_ms"] <= 1.05 * t["walk_kernel_ms"] + 0.05
    assert t["span_ms"] > 0.0


def test_option_api(gpu_available):
    """wost_set_option / wost_get_option / wost_options_report on a handle: unknown names and
    out-of-range values raise ValueError, study-build-only names NotImplementedError in the
    product library; a kernel option rebuilds the handle's kernel and changes no bits."""
    sc = _scenario("poisson_square")
    s = sc.solver(device=0)
    assert s.options_report()["build"] == "product" and _set_options(s) == {}
    with pytest.raises(ValueError, match="unknown option"):
        s.set_option("no_such_option", 1)
    with pytest.raises(ValueError, match="out of range"):
        s.set_option("pool_slots", 0)
    with pytest.raises(ValueError):
        s.set_option("walk_block", 100)          # whole waves only
    with pytest.raises(NotImplementedError, match="study builds only"):
        s.set_option("exp_flags", 32)
    pts = np.ascontiguousarray(sc.points[:4], np.float32)
    ref = _walks(s, pts, 500, sc, seed=3)
    s.set_option("walk_block", 512)
    assert s.get_option("walk_block") == 512.0
    got = _walks(s, pts, 500, sc, seed=3)
    assert s.last_timing["block_threads"] == 512
    assert _set_options(s) == {"walk_block": 512}
    np.testing.assert_array_equal(got[0], ref[0])
    np.testing.assert_array_equal(got[1], ref[1])
