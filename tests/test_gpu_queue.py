"""The walk kernels' work queue and launch shape (wost_walk.h refill, wost_api.hip
solve_impl): a walk's result depends only on its id, so every queue shape gives the
same bits. The shape follows the handle's previous solve (round 5): after short walks
(< 32 steps) the waves start with static 64-walk chunks and the grid holds ~4 walks per
lane; the dynamic chunk's floor is 1024 / (previous mean steps); the block reduce resets
the queue head for the next launch. Each case solves the same problem on a fresh handle
(no previous solve) and on a handle whose previous solve set another shape, and compares
the per-walk values and step counts bit for bit.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _walks(s, pts, W, sc, seed):
    v, st = s.solve_walks(pts, nWalks=W, maxSteps=sc.max_steps, eps=sc.eps, seed=seed)
    return np.asarray(v).view(np.uint32).copy(), np.asarray(st).copy()


@pytest.mark.parametrize("name, big, small", [
    ("poisson_square", (64, 4000), (3, 100)),       # short walks: static chunks, fewer workgroups
    ("poisson_square", (64, 4000), (64, 3000)),     # ... with dynamic chunks after the static ones
    ("dcr_dipole", (48, 2000), (5, 300)),           # long walks with a Neumann boundary: chunk floor from 76 steps
])
def test_queue_shape_changes_no_bits(gpu_available, name, big, small):
    from dcrmontecarlo_amd import scenarios as S

    sc = S.ALL[name](**({"n_walks": 1} if name == "dcr_dipole" else {}))
    pts_big = np.resize(sc.points, (big[0], 2)).astype(np.float32)
    pts_small = np.ascontiguousarray(pts_big[:small[0]])
    fresh = sc.solver(device=0)
    ref = _walks(fresh, pts_small, small[1], sc, seed=7)      # no previous solve
    warm = sc.solver(device=0)
    _walks(warm, pts_big, big[1], sc, seed=3)                 # sets the handle's walk length
    got = _walks(warm, pts_small, small[1], sc, seed=7)
    again = _walks(warm, pts_small, small[1], sc, seed=7)     # the queue head reset by the reduce
    for g in (got, again):
        np.testing.assert_array_equal(g[1], ref[1])
        np.testing.assert_array_equal(g[0], ref[0])
    assert ref[1].sum() > 0


def test_static_chunks_cover_every_walk(gpu_available):
    """Fewer walks than one static chunk per wave (the queue is never dequeued): every walk
    runs once -- the step counts of a tiny solve after short walks equal a fresh handle's."""
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
