"""Walk-range shards and libwost's RCCL path on one GPU.

wost_solve_range must reproduce, block for block and bit for bit, the blocks of
the full solve it is a shard of; wost_solve_distributed on a one-rank
communicator must equal wost_solve bit for bit. RCCL cannot put two ranks on one
GPU, so the R > 1 path of wost_solve_distributed -- its C++ protocol
wost_distributed_run (agreement all-reduce, padded all-gather, ordered merge) --
runs here with R threads as ranks on real device shards (R = 2, 3, 8; single- and
multi-source rows), and over gloo with oracle shards in test_distributed.py.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

B = 4096   # WOST_BLOCK_WALKS


def _solver(name):
    from dcrmontecarlo_amd import scenarios as S

    sc = S.ALL[name]()
    return sc, sc.solver(device=0)


@pytest.mark.parametrize("name", ["dcr_dipole", "variable_coefficients", "poisson_square"])
def test_walk_ranges_equal_the_full_solves_blocks(gpu_available, name):
    sc, s = _solver(name)
    pts = sc.points[:5]
    W = 3 * B + 1000
    nbpp = 4
    full = s.solve_blocks(pts, W, 0, len(pts) * nbpp, sc.max_steps, sc.eps, seed=21).reshape(len(pts), nbpp, 3)
    for w0, w1 in [(0, B), (B, 3 * B), (3 * B, W), (B, W), (0, W)]:
        part = s.solve_range(pts, W, w0, w1, sc.max_steps, sc.eps, seed=21)
        assert np.array_equal(part, full[:, w0 // B:(w1 + B - 1) // B]), (w0, w1)
    # per-walk values of a range are the full solve's walks of that range
    v, st = s.solve_walks(pts, nWalks=W, maxSteps=sc.max_steps, eps=sc.eps, seed=21)
    from dcrmontecarlo_amd import _lib

    vr = np.empty(len(pts) * (W - B), np.float32)
    sr = np.empty(len(pts) * (W - B), np.uint32)
    _lib.check(_lib.lib.wost_solve_range(s._h, _lib.fptr(np.ascontiguousarray(pts, np.float32)), len(pts), W, B, W,
                                         sc.max_steps, sc.eps, 21, None, None, _lib.fptr(vr), _lib.u32ptr(sr)))
    assert np.array_equal(vr.reshape(len(pts), -1), v[:, B:]) and np.array_equal(sr.reshape(len(pts), -1), st[:, B:])


def test_walk_range_rejects_unaligned_ends(gpu_available):
    sc, s = _solver("laplace_square")
    with pytest.raises(ValueError):
        s.solve_range(sc.points[:2], 3 * B, 100, 2 * B, sc.max_steps, sc.eps)
    with pytest.raises(ValueError):
        s.solve_range(sc.points[:2], 3 * B, B, B + 7, sc.max_steps, sc.eps)
    with pytest.raises(ValueError):
        s.solve_range(sc.points[:2], 3 * B, 2 * B, B, sc.max_steps, sc.eps)


def test_walk_range_longer_than_one_launch(gpu_available):
    """A range of more than 2^26 walks of a point is solved as sub-ranges: same blocks."""
    sc, s = _solver("laplace_square")
    pts = sc.points[:1]
    W = (1 << 26) + 3 * B + 5
    nbpp = -(-W // B)
    full = s.solve_blocks(pts, W, 0, nbpp, sc.max_steps, sc.eps, seed=4).reshape(1, nbpp, 3)
    part = s.solve_range(pts, W, B, W, sc.max_steps, sc.eps, seed=4)
    assert part.shape == (1, nbpp - 1, 3)
    assert np.array_equal(part, full[:, 1:])
    assert s.last_timing["n_launches"] >= 2


def test_multi_source_walk_ranges(gpu_available):
    """Range shards of a multi-source handle carry 2S+1 columns and equal the full blocks."""
    from dcrmontecarlo_amd import _lib
    from dcrmontecarlo_amd import survey  # noqa: F401  (scenario helpers)
    import ctypes

    sc, s = _solver("dcr_dipole")
    pts = sc.points[10:14]
    W = 2 * B + 77
    srcs = [sc.f, 2.0 * sc.f, 0.5 * sc.f]
    packed = [_lib.make_field(s._conv(f, "src")) for f in srcs]
    arr = (ctypes.POINTER(_lib.WostField) * 3)(*[ctypes.pointer(wf) for wf, _ in packed])
    _lib.check(_lib.lib.wost_set_sources(s._h, arr, 3))
    nb = len(pts) * 3
    full = np.zeros((nb, 7))
    _lib.check(_lib.lib.wost_solve_multi(s._h, _lib.fptr(np.ascontiguousarray(pts)), len(pts), W, 0, nb, sc.max_steps,
                                         sc.eps, 8, _lib.dptr(full), None, None, None))
    full = full.reshape(len(pts), 3, 7)
    part = s.solve_range(pts, W, B, W, sc.max_steps, sc.eps, seed=8)
    assert part.shape == (len(pts), 2, 7)
    assert np.array_equal(part, full[:, 1:])


@pytest.mark.parametrize("name", ["dcr_dipole", "notebook_dcr"])
def test_solve_distributed_one_rank_equals_solve(gpu_available, name):
    """wost_solve_distributed over a one-rank RCCL communicator: bitwise the one-GPU solve."""
    from dcrmontecarlo_amd import comm

    sc, s = _solver(name)
    pts = sc.points[:12]
    W = 5 * B + 123
    u, st = s.solve(pts, nWalks=W, maxSteps=sc.max_steps, eps=sc.eps, seed=77, return_stats=True)
    c = comm.Communicator(comm.unique_id(), 1, 0, 0)
    try:
        ud, std, t = comm.solve_distributed(s, c, pts, W, sc.max_steps, sc.eps, seed=77)
        assert np.array_equal(ud, u)
        assert np.array_equal(std.mean, st.mean) and np.array_equal(std.stderr, st.stderr)
        assert t["all_steps"] == st.total_steps and (t["walk_begin"], t["walk_end"]) == (0, W)
        g = c.allgather(np.arange(5.0))
        assert g.shape == (1, 5) and np.array_equal(g[0], np.arange(5.0))
        assert float(c.allreduce([3.0], "max")[0]) == 3.0
        c.barrier()
    finally:
        c.close()


def test_shards_of_a_solve_merge_to_the_solve(gpu_available):
    """What each rank of an R-rank wost_solve_distributed computes -- its walk range of every
    point, solved on the device -- goes through libwost's own protocol (wost_distributed_run,
    R threads as ranks): the merged point sums equal the one-GPU sums bit for bit on every
    rank (R = 2, 3, 8), with the host mirror agreeing."""
    from dcrmontecarlo_amd import distributed as D
    from rank_threads import RankThreads

    sc, s = _solver("dcr_dipole")
    pts = sc.points[:6]
    W = 9 * B + 5
    sums = s.solve_blocks(pts, W, 0, s.num_blocks(len(pts), W), sc.max_steps, sc.eps, seed=3)
    one = D.point_sums(sums, len(pts))
    for R in (2, 3, 8):
        shards = {}
        for r in range(R):   # the device solves, one after another
            w0, w1 = D.shard_walk_range(W, R, r)
            shards[(w0, w1)] = s.solve_range(pts, W, w0, w1, sc.max_steps, sc.eps, seed=3) if w1 > w0 else None
        res = RankThreads(R).run(lambda r, ar, ag: D.run_protocol(R, r, len(pts), W, 3,
                                                                  lambda w0, w1: shards[(w0, w1)], ar, ag))
        for r in range(R):
            assert not isinstance(res[r], Exception), res[r]
            assert np.array_equal(res[r][0], one), R
            assert res[r][1] == D.shard_walk_range(W, R, r)
            assert res[r][2] == int(one[:, 2].sum())


def test_multi_source_shards_merge_through_the_protocol(gpu_available):
    """Multi-source rows (2S+1 = 7) through wost_distributed_run with R = 3 thread ranks:
    equal to one-GPU solve_sources bit for bit; and comm.solve_sources_distributed on a
    one-rank RCCL communicator equals solve_sources."""
    from dcrmontecarlo_amd import comm
    from dcrmontecarlo_amd import distributed as D
    from rank_threads import RankThreads

    sc, s = _solver("dcr_dipole")
    pts = sc.points[10:14]
    W = 4 * B + 77
    srcs = [sc.f, 2.0 * sc.f, 0.5 * sc.f]
    u1, st1 = s.solve_sources(pts, srcs, nWalks=W, maxSteps=sc.max_steps, eps=sc.eps, seed=8, return_stats=True)
    fields = s.source_fields(srcs)
    R = 3
    with s.sources_installed(fields):
        shards = {D.shard_walk_range(W, R, r): s.solve_range(pts, W, *D.shard_walk_range(W, R, r), sc.max_steps,
                                                              sc.eps, seed=8) for r in range(R)}
    res = RankThreads(R).run(lambda r, ar, ag: D.run_protocol(R, r, len(pts), W, 7, lambda a, b: shards[(a, b)],
                                                              ar, ag))
    for r in range(R):
        sums = res[r][0]
        for k in range(3):
            assert np.array_equal(sums[:, 2 * k] / W, st1.mean[k])
    c = comm.Communicator(comm.unique_id(), 1, 0, 0)
    try:
        ud, std, t = comm.solve_sources_distributed(s, c, pts, srcs, W, sc.max_steps, sc.eps, seed=8)
        assert np.array_equal(ud, u1) and np.array_equal(std.stderr, st1.stderr)
        assert t["all_steps"] == st1.total_steps
        with pytest.raises(ValueError):
            with s.sources_installed(fields):
                comm.solve_distributed(s, c, pts, W, sc.max_steps, sc.eps, seed=8)
        with pytest.raises(ValueError):
            c.allreduce([1.0], "min")
    finally:
        c.close()


def test_wenner_survey_through_communicators_equals_one_gpu(gpu_available):
    """The C5 survey's multi-GPU path (survey.run_wenner_survey(comm=...): both fields'
    walk-range solves concurrent, every collective of libwost's protocol issued from
    one thread in a fixed order) on a one-rank RCCL communicator equals the one-GPU
    survey bit for bit (reduced: 24 electrodes, 2,000-segment topography), with the
    fields concurrent or not; a communicator pair is refused."""
    from dcrmontecarlo_amd import comm
    from dcrmontecarlo_amd import scenarios as S
    from dcrmontecarlo_amd import survey

    sc = S.wenner_topography(n_electrodes=24, n_walks=2 * B + 11, n_segments=2000)
    sm = sc.solver(device=0)
    sh = survey.homogeneous_solver(sc, 1e-2, sm, device=0)
    ref = survey.run_wenner_survey(sc, 1e-2, sc.n_walks, seed=3, solvers=(sm, sh), concurrent=False)
    cs = [comm.Communicator(comm.unique_id(), 1, 0, 0) for _ in range(2)]
    try:
        for concurrent in (True, False):
            got = survey.run_wenner_survey(sc, 1e-2, sc.n_walks, seed=3, solvers=(sm, sh), comm=cs[0],
                                           concurrent=concurrent)
            for a, b in ((got.model, ref.model), (got.background, ref.background)):
                assert np.array_equal(a.dv, b.dv) and np.array_equal(a.se, b.se)
            assert np.array_equal(got.rho.rho_a, ref.rho.rho_a, equal_nan=True)
            assert got.walk_steps == got.local_walk_steps == ref.walk_steps
        with pytest.raises(ValueError, match="one communicator"):
            survey.run_wenner_survey(sc, 1e-2, sc.n_walks, seed=3, solvers=(sm, sh), comm=(cs[0], cs[1]))
    finally:
        for c in cs:
            c.close()
