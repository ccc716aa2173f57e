"""The multi-GPU Wenner survey's collective order (survey._run_fields_distributed), on
CPU: thread ranks (tests/rank_threads.py) drive libwost's real protocol
(wost_distributed_run) with solvers whose walk-range block rows are a deterministic
function of the global block, so that an R-rank survey must equal the one-rank survey
bit for bit. Every rank must issue the same collectives in the same order -- group by
group, model before background -- although each rank's two fields solve concurrently
in their own threads, and a failure on one rank must reach every rank."""
import contextlib
import threading
import time

import numpy as np
import pytest

from rank_threads import RankThreads

B = 4096   # WOST_BLOCK_WALKS


class FakeSolver:
    """solve_range / solve_sources of a solver whose block k of point p under source s
    has the rows (sum, sum^2, steps) = f(seed, p, k, s): the device's block sums stand-in.
    ``jitter`` sleeps a random while per solve, so the two fields' threads finish their
    groups in varying order."""

    def __init__(self, tag, jitter=0.0, fail_group=None, seed=0):
        self.tag, self.jitter, self.fail_group = float(tag), jitter, fail_group
        self.rng = np.random.default_rng(seed)
        self.S = 1
        self.last_timing = {}
        self.lock = threading.Lock()

    def source_fields(self, srcs):
        return list(srcs)

    @contextlib.contextmanager
    def sources_installed(self, fields):
        self.S = len(fields)
        yield self.S
        self.S = 1

    def _blocks(self, points, seed, k0, k1):
        p = np.asarray(points, np.float64)
        k = np.arange(k0, k1, dtype=np.float64)
        n, nb, S = p.shape[0], k1 - k0, self.S
        rows = np.zeros((n, nb, 2 * S + 1))
        base = (p[:, 0:1] * 0.37 + p[:, 1:2] * 1.3 + self.tag + (seed % 1000) * 1e-3)[:, :, None]
        for s in range(S):
            x = np.sin(base[:, :, 0] * (s + 1) + k[None, :] * 0.61) * 1e3 + 1e-7 * k[None, :]
            rows[:, :, 2 * s] = x
            rows[:, :, 2 * s + 1] = x * x + 1e6
        rows[:, :, -1] = 4096.0 * (3 + (k[None, :] % 5)) + 0 * base[:, :, 0]
        return rows

    def _sleep(self):
        if self.jitter:
            with self.lock:
                d = float(self.rng.random()) * self.jitter
            time.sleep(d)

    def solve_range(self, points, nWalks, w0, w1, maxSteps, eps, seed):
        self._sleep()
        if self.fail_group is not None and seed == self.fail_group:
            raise RuntimeError("injected local failure")
        rows = self._blocks(points, seed, w0 // B, -(-w1 // B))
        self.last_timing = {"total_steps": int(rows[:, :, -1].sum()), "walk_kernel_ms": 1.0, "total_ms": 1.0}
        return rows

    def solve_sources(self, points, srcs, nWalks, maxSteps, eps, seed, return_stats=True):
        from dcrmontecarlo_amd.solvers.WoStSolver import SolveStats, _stats_of_multi

        self._sleep()
        with self.sources_installed(srcs):
            rows = self._blocks(points, seed, 0, -(-int(nWalks) // B))
        acc = np.zeros((rows.shape[0], rows.shape[2]))
        for b in range(rows.shape[1]):      # block order, from 0.0: the one-GPU point sums
            acc += rows[:, b]
        stats = _stats_of_multi(acc, int(nWalks))
        st = SolveStats(mean=np.stack([x.mean for x in stats]), stderr=np.stack([x.stderr for x in stats]),
                        mean_steps=stats[0].mean_steps, walks=int(nWalks), total_steps=int(acc[:, -1].sum()),
                        kernel_ms=1.0, total_ms=1.0)
        return None, st


class LoggedComm:
    def __init__(self, rank, n_ranks, allreduce, allgather):
        self.rank, self.n_ranks, self._ar, self._ag, self.log = rank, n_ranks, allreduce, allgather, []

    def allreduce(self, a, op="sum"):
        self.log.append(("allreduce", op, int(np.size(a))))
        return self._ar(np.asarray(a, np.float64), op)

    def allgather(self, a):
        self.log.append(("allgather", int(np.size(a))))
        return self._ag(np.asarray(a, np.float64))


def _scenario():
    from dcrmontecarlo_amd import scenarios as S

    return S.wenner_topography(n_electrodes=40, n_walks=1, n_segments=64)


def _seed_of_group(g, seed=5):
    from dcrmontecarlo_amd import survey

    return survey.group_seed(seed, g)


@pytest.mark.parametrize("R,walks,pairs", [(2, 3 * B + 100, 1), (3, 5 * B, 1), (2, B // 2, 1), (2, 3 * B + 100, 2),
                                           (3, 5 * B, 3)])
def test_distributed_survey_equals_one_rank_with_one_collective_order(R, walks, pairs):
    """... with `pairs` (model, background) handle pairs per rank: 2 x pairs worker
    threads solve concurrently, the collective order stays the same."""
    from dcrmontecarlo_amd import survey

    sc = _scenario()
    one = survey.run_wenner_survey(sc, 1e-2, walks, seed=5, solvers=(FakeSolver(0.0), FakeSolver(0.5)))
    many = survey.run_wenner_survey(sc, 1e-2, walks, seed=5,
                                    solvers=sum(((FakeSolver(0.0, 0.005, seed=p), FakeSolver(0.5, 0.005, seed=7 + p))
                                                 for p in range(pairs)), ()))
    np.testing.assert_array_equal(many.model.dv, one.model.dv)
    np.testing.assert_array_equal(many.background.se, one.background.se)
    assert many.walk_steps == one.walk_steps
    rt = RankThreads(R)
    comms = {}

    def body(r, ar, ag):
        c = comms[r] = LoggedComm(r, R, ar, ag)
        sv = sum(((FakeSolver(0.0, 0.01, seed=10 * r + p), FakeSolver(0.5, 0.01, seed=9 + 10 * r + p))
                  for p in range(pairs)), ())
        return survey.run_wenner_survey(sc, 1e-2, walks, seed=5, comm=c, solvers=sv)

    res = rt.run(body)
    for r in range(R):
        assert not isinstance(res[r], Exception), res[r]
        for got, want in ((res[r].model, one.model), (res[r].background, one.background)):
            np.testing.assert_array_equal(got.dv, want.dv)
            np.testing.assert_array_equal(got.se, want.se)
        assert res[r].walk_steps == one.walk_steps
        # the protocol's per-rank phases (bench.py's per_rank breakdown), summed over groups
        ph = res[r].phase_ms
        assert set(ph) == {"wait_ms", "agree_ms", "gather_ms", "merge_ms"} and min(ph.values()) >= 0.0
        assert ph["agree_ms"] > 0.0
    assert one.phase_ms is None
    # one collective sequence on every rank: per group, model then background, each an
    # agreement all-reduce (41 numbers) and -- when some rank holds walks -- one all-gather
    G = len(list(survey.wenner_batches(40, 1)))
    logs = [comms[r].log for r in range(R)]
    assert all(lg == logs[0] for lg in logs)
    ag = [e for e in logs[0] if e[0] == "allreduce"]
    assert len(ag) == 2 * G and all(e == ("allreduce", "max", 41) for e in ag)   # wost_distributed_run agreement
    assert sum(e[0] == "allgather" for e in logs[0]) == 2 * G
    sizes = [e[1] for e in logs[0] if e[0] == "allgather"]
    assert sizes[0::2] == sizes[1::2]       # model and background of a group gather alike


def test_distributed_survey_failure_on_one_rank_reaches_every_rank():
    from dcrmontecarlo_amd import survey

    sc = _scenario()
    R = 2
    rt = RankThreads(R)
    bad = _seed_of_group(2)

    def body(r, ar, ag):
        c = LoggedComm(r, R, ar, ag)
        return survey.run_wenner_survey(sc, 1e-2, 3 * B, seed=5, comm=c,
                                        solvers=(FakeSolver(0.0, 0.005, fail_group=bad if r == 1 else None),
                                                 FakeSolver(0.5, 0.005)))

    t0 = time.time()
    res = rt.run(body)
    assert time.time() - t0 < 60
    assert isinstance(res[1], RuntimeError) and "injected" in str(res[1])
    assert isinstance(res[0], Exception) and "another rank failed" in str(res[0])


def test_survey_refuses_a_communicator_pair_and_odd_handles():
    from dcrmontecarlo_amd import survey

    with pytest.raises(ValueError, match="one communicator"):
        survey.run_wenner_survey(_scenario(), 1e-2, 16, comm=(object(), object()),
                                 solvers=(FakeSolver(0.0), FakeSolver(0.5)))
    with pytest.raises(ValueError, match="pairs"):
        survey.run_wenner_survey(_scenario(), 1e-2, 16, solvers=(FakeSolver(0.0), FakeSolver(0.5), FakeSolver(1.0)))


def test_bench_rank_breakdown_over_thread_ranks():
    """bench.py's per_rank block (VERDICT r04 missing #3): every rank's timed-region
    figures all-gathered, min / max / mean per figure and the kernel's max/mean."""
    import bench

    R = 3
    rt = RankThreads(R)

    def body(r, ar, ag):
        c = LoggedComm(r, R, ar, ag)
        return bench.rank_breakdown(c, {"elapsed_ms": 100.0 + r, "kernel_ms": 50.0 + 10 * r, "local_ms": 60.0 + r,
                                        "agree_ms": 5.0 - r, "gather_ms": 1.0, "merge_ms": 0.25,
                                        "walk_steps": 1000 * (r + 1)})

    res = rt.run(body)
    for r in range(R):
        b = res[r]
        assert not isinstance(b, Exception), b
        assert b["ranks"] == R
        assert b["kernel_ms"] == {"min": 50.0, "max": 70.0, "mean": 60.0, "max_over_mean": 70.0 / 60.0}
        assert b["walk_steps"]["min"] == 1000 and b["walk_steps"]["max"] == 3000
        assert b["agree_ms"]["min"] == 3.0 and b["elapsed_ms"]["max"] == 102.0
        assert all(v["min"] <= v["mean"] <= v["max"] for k, v in b.items() if k != "ranks")
