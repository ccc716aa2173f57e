"""DCR survey layer: electrode arrays, potential differences, apparent resistivity.

CPU tests cover the host arithmetic (and the oracle's own homogeneous survey);
the GPU test runs a reduced dcr_dipole survey on the device and compares rho_a
with the CPU oracle on the same walks (same seeds).
"""
import numpy as np
import pytest

from dcrmontecarlo_amd import scenarios as S
from dcrmontecarlo_amd import survey


def test_dipole_dipole_pairs_adjacent():
    p = survey.dipole_dipole_pairs(5)
    assert p.tolist() == [[0, 1], [1, 2], [2, 3], [3, 4]]
    assert survey.dipole_dipole_pairs(1).shape == (0, 2)


def test_wenner_quadripoles():
    q = survey.wenner_quadripoles(8, a=2)
    assert q.tolist() == [[0, 2, 4, 6], [1, 3, 5, 7]]
    assert survey.wenner_quadripoles(3, a=1).shape == (0, 4)


@pytest.mark.parametrize("E,a", [(256, 1), (256, 5), (40, 1), (7, 2), (16, 1)])
def test_wenner_batches_walk_each_receiver_once(E, a):
    """Multi-source batching of a Wenner line: each of a quadripole's receivers M and N is
    solved in a group holding its transmitter, at most 16 transmitters per group, and
    every electrode belongs to one group (walked once per field)."""
    groups = list(survey.wenner_batches(E, a))
    seen = []
    for j0, j1, t0, t1 in groups:
        assert 0 < t1 - t0 <= 16 and 0 <= j0 < j1 <= E
        seen.extend(range(j0, j1))
    assert len(seen) == len(set(seen))
    for q, (A, M, N, B) in enumerate(survey.wenner_quadripoles(E, a)):
        for e in (M, N):
            assert any(j0 <= e < j1 and t0 <= q < t1 for j0, j1, t0, t1 in groups), (q, e)


def test_paired_rho_a_and_replicas():
    """Common random numbers: identical model and background walks give rho_bg with a zero
    error; the replicas and matched-walk p-values behave on known inputs."""
    rng = np.random.default_rng(0)
    h = rng.exponential(size=(4, 800)) * np.array([[4.0], [3.0], [2.0], [1.0]])
    pairs = survey.dipole_dipole_pairs(4)
    r = survey.paired_apparent_resistivity(h, h, pairs, 0.01)
    np.testing.assert_allclose(r.rho_a, 0.01)
    np.testing.assert_allclose(r.se, 0.0, atol=1e-9)
    assert r.resolved.all()
    m = 2.0 * h                                        # a uniformly doubled response: rho_a = 2 rho_bg
    r2 = survey.paired_apparent_resistivity(m, h, pairs, 0.01)
    np.testing.assert_allclose(r2.rho_a, 0.02)
    rep = survey.replica_rho_a(m, h, pairs, 0.01, 100)
    assert rep.shape == (8, 3)
    np.testing.assert_allclose(rep, 0.02)
    p = survey.matched_walk_pvalues(rep, np.array([0.02, 0.03, 0.01]))
    assert p.tolist() == [1.0, 0.0, 0.0]


def test_potential_differences_and_errors():
    u = np.array([3.0, 1.0, 0.5])
    se = np.array([0.3, 0.4, 0.0])
    d = survey.potential_differences(u, se, survey.dipole_dipole_pairs(3))
    np.testing.assert_allclose(d.dv, [2.0, 0.5])
    np.testing.assert_allclose(d.se, [0.5, 0.4])


def test_apparent_resistivity_of_background_is_rho_bg():
    d = survey.DipoleData(np.array([2.0, -1.0, 1e-9]), np.array([0.01, 0.01, 0.01]))
    r = survey.apparent_resistivity(d, d, 0.01)
    np.testing.assert_allclose(r.rho_a, 0.01)
    assert r.resolved.tolist() == [True, True, False]


def test_apparent_resistivity_error_propagation():
    m = survey.DipoleData(np.array([2.0]), np.array([0.2]))
    h = survey.DipoleData(np.array([1.0]), np.array([0.1]))
    r = survey.apparent_resistivity(m, h, 0.5)
    assert r.rho_a[0] == pytest.approx(1.0)
    assert r.se[0] == pytest.approx(1.0 * np.sqrt(0.1 ** 2 + 0.1 ** 2))


def test_compare_uses_jointly_resolved_dipoles():
    a = survey.ApparentResistivity(np.array([1.0, 2.0, 5.0]), np.array([0.1, 0.1, 0.1]),
                                   np.array([True, True, False]))
    b = survey.ApparentResistivity(np.array([1.1, 1.9, 0.0]), np.array([0.2, 0.2, 0.2]),
                                   np.array([True, True, True]))
    c = survey.compare(a, b)
    assert c["resolved"] == 2
    assert c["rmse"] == pytest.approx(0.1)
    assert c["mc_1sigma"] == pytest.approx(0.2)
    none = survey.compare(a, survey.ApparentResistivity(b.rho_a, b.se, np.zeros(3, bool)))
    assert none == {"rmse": None, "mc_1sigma": None, "resolved": 0, "z_rms": None, "z_max": None}
    assert c["z_max"] == pytest.approx(0.1 / np.sqrt(0.05))
    assert c["z_rms"] == pytest.approx(0.1 / np.sqrt(0.05))


def test_homogeneous_scenario_keeps_survey():
    sc = S.dcr_dipole(n_electrodes=6, n_walks=10)
    h = survey.homogeneous(sc, 100.0)
    assert h.alpha.pack()[0] and h.f is sc.f and h.neumann is sc.neumann
    np.testing.assert_array_equal(h.points, sc.points)
    assert float(h.alpha(np.array([1.0, -30.0]))) == pytest.approx(100.0)


@pytest.mark.gpu
def test_gpu_survey_rho_a_matches_cpu_oracle(gpu_available):
    """Reduced C4 survey (12 electrodes around the sources x 16000 walks): rho_a on
    the GPU vs the CPU oracle on the same walks. The walks agree one for one up to
    the scenario's chaos (~1-2% diverge), so the rho_a RMSE is a small fraction of
    the Monte-Carlo 1-sigma (the north-star bound is RMSE <= 1 sigma)."""
    from oracle import oracle as O

    sc = S.dcr_dipole(n_electrodes=48, n_walks=16000)
    sc.points = sc.points[18:30]          # x = -16.5 .. 16.5: around the two sources
    alpha_bg = 100.0
    res = survey.run_dipole_dipole(sc, alpha_bg, sc.n_walks, seed=5, device=0)
    sm, sh = sc.solver(device=0), survey.homogeneous(sc, alpha_bg).solver(device=0)
    cm = O.Problem.from_scenario(sc, sigma_bar=sm.sigma_bar).solve(sc.points, sc.n_walks, sc.max_steps, sc.eps, 5)
    ch = O.Problem.from_scenario(survey.homogeneous(sc, alpha_bg), sigma_bar=sh.sigma_bar).solve(
        sc.points, sc.n_walks, sc.max_steps, sc.eps, 5)
    pairs = survey.dipole_dipole_pairs(len(sc.points))
    rc = survey.apparent_resistivity(survey.potential_differences(cm[0], cm[1], pairs),
                                     survey.potential_differences(ch[0], ch[1], pairs), 1.0 / alpha_bg)
    c = survey.compare(res.rho, rc)
    assert c["resolved"] >= 4, c
    assert c["rmse"] <= 0.5 * c["mc_1sigma"], c
    # the background survey's own rho_a vs the model's is a different quantity: the
    # resistive/conductive bodies must move rho_a away from rho_bg somewhere
    assert np.nanmax(np.abs(res.rho.rho_a[res.rho.resolved] - 0.01)) > 0.0


def test_dipole_dipole_quadripoles():
    q = survey.dipole_dipole_quadripoles(6, n_max=2)
    assert q.tolist() == [[0, 1, 2, 3], [0, 1, 3, 4], [1, 2, 3, 4], [1, 2, 4, 5], [2, 3, 4, 5]]
    assert survey.dipole_dipole_quadripoles(3).shape == (0, 4)


def test_dipole_source_is_antisymmetric_and_normalised():
    f = survey.dipole_source((-3.0, 0.0), (3.0, 0.0), 0.5)
    x = np.linspace(-8, 8, 641)
    X, Y = np.meshgrid(x, x)
    v = f(np.stack([X.ravel(), Y.ravel()], 1)).reshape(X.shape)
    v = np.asarray(v, np.float64)
    np.testing.assert_allclose(v, -v[:, ::-1], atol=1e-6)
    h = x[1] - x[0]
    pos = np.where(X < 0, v, 0).sum() * h * h
    assert pos == pytest.approx(1.0, rel=1e-3)


class _FakeSolver:
    """solve_sources stand-in: u_k(x) = a k-dependent linear function of the point, so the
    survey's group/transmitter bookkeeping can be checked on the host."""

    sigma_bar = 10.0

    def __init__(self, scale):
        self.scale = scale
        self.calls = []

    def values(self, pts, srcs):
        k = np.array([float(np.asarray(s(np.array([0.0, -50.0])))) for s in srcs])   # identifies the source
        return self.scale * (k[:, None] * 1e3 + pts[:, 0][None, :])

    def solve_sources(self, pts, srcs, nWalks, maxSteps, eps, seed, return_stats):
        from dcrmontecarlo_amd.solvers.WoStSolver import SolveStats

        self.calls.append((len(pts), len(srcs), seed))
        u = self.values(np.asarray(pts), srcs)
        st = SolveStats(mean=u, stderr=np.full_like(u, 1e-6), mean_steps=np.ones(len(pts)), walks=nWalks,
                        total_steps=len(pts) * nWalks, kernel_ms=1.0, total_ms=1.0)
        return u.astype(np.float32), st


@pytest.mark.parametrize("E,a", [(40, 1), (23, 2)])
def test_wenner_survey_bookkeeping_one_gpu(E, a):
    """run_wenner_survey on host stand-ins: every quadripole's dV is u_q(M) - u_q(N) of
    its own transmitter, and each group is solved once per field with its own seed."""
    sc = S.wenner_topography(n_electrodes=E, n_walks=8, n_segments=100)
    Q = E - 3 * a
    srcs = [survey.dipole_source(sc.points[q], sc.points[q + 3 * a], 0.5) for q in range(Q)]
    fm, fh = _FakeSolver(1.0), _FakeSolver(0.5)
    r1 = survey.run_wenner_survey(sc, 1e-2, 8, a=a, seed=3, solvers=(fm, fh), concurrent=False)
    groups = list(survey.wenner_batches(E, a))
    assert len(fm.calls) == len(fh.calls) == len(groups) == r1.launches
    assert len({c[2] for c in fm.calls}) == len(groups)            # a seed per group
    assert [c[2] for c in fm.calls] == [c[2] for c in fh.calls]    # common random numbers
    quad = survey.wenner_quadripoles(E, a)
    for q, (A, M, N, B) in enumerate(quad):
        u = fm.values(sc.points[[M, N]], [srcs[q]])[0]
        assert r1.model.dv[q] == pytest.approx(u[0] - u[1], rel=1e-12)
    np.testing.assert_allclose(r1.rho.rho_a, 1e2 * 2.0)
    assert r1.walk_steps == r1.local_walk_steps == 2 * E * 8

    # the communicator path (walk-range shards, one fixed collective order) runs the real
    # protocol over thread ranks in tests/test_survey_distributed.py


class _PreparingSolver(_FakeSolver):
    """A stand-in that also records wost_prepare_sources calls (from the prepare pool)."""

    def __init__(self, scale, log, name):
        super().__init__(scale)
        self.log, self.name = log, name

    def prepare_sources(self, srcs, n_points):
        k = tuple(float(np.asarray(s(np.array([0.0, -50.0])))) for s in srcs)
        self.log.append((self.name, k, n_points))


def test_wenner_survey_prepares_every_group_kernel_once():
    """survey.prepare_survey_kernels: before the first survey's solves, every group's kernel
    of each field is prepared on the handle that solves it (group g on pair g mod k), with
    the group's transmitters and electrode count; a second survey on the same solvers
    prepares nothing."""
    E = 40
    sc = S.wenner_topography(n_electrodes=E, n_walks=8, n_segments=100)
    log = []
    sv = (_PreparingSolver(1.0, log, "m0"), _PreparingSolver(0.5, log, "h0"),
          _PreparingSolver(1.0, log, "m1"), _PreparingSolver(0.5, log, "h1"))
    survey.run_wenner_survey(sc, 1e-2, 8, seed=3, solvers=sv)
    groups = list(survey.wenner_batches(E, 1))
    srcs = [survey.dipole_source(sc.points[q], sc.points[q + 3], 0.5) for q in range(E - 3)]
    want = set()
    for g, (j0, j1, t0, t1) in enumerate(groups):
        k = tuple(float(np.asarray(s(np.array([0.0, -50.0])))) for s in srcs[t0:t1])
        for f, name in enumerate(("m", "h")):
            want.add((f"{name}{g % 2}", k, j1 - j0))
    assert len(log) == 2 * len(groups) and set(log) == want
    survey.run_wenner_survey(sc, 1e-2, 8, seed=4, solvers=sv)
    assert len(log) == 2 * len(groups)                              # already prepared
    sc2 = S.wenner_topography(n_electrodes=E - 4, n_walks=8, n_segments=100)
    survey.run_wenner_survey(sc2, 1e-2, 8, seed=4, solvers=sv)     # other electrodes: prepared again
    assert len(log) == 2 * len(groups) + 2 * len(list(survey.wenner_batches(E - 4, 1)))


def test_apparent_resistivity_resolves_only_with_the_model_error_small():
    """resolved needs the model's dV resolved too (round-2 verdict): a precise background
    with a model dV inside its own noise is not a resolved rho_a."""
    h = survey.DipoleData(np.array([1.0, 1.0]), np.array([1e-3, 1e-3]))
    m = survey.DipoleData(np.array([0.5, 0.5]), np.array([0.01, 1.0]))
    r = survey.apparent_resistivity(m, h, 100.0)
    assert r.resolved.tolist() == [True, False]


def test_physical_wenner_variant_drops_only_the_air_term():
    lit = S.wenner_topography(n_electrodes=8, n_walks=1, n_segments=100)
    phys = S.wenner_topography_physical(n_electrodes=8, n_walks=1, n_segments=100)
    assert phys.name == "wenner_topography_physical" and np.array_equal(phys.points, lit.points)
    below = np.array([[0.0, -300.0], [-120.0, -80.0], [120.0, -80.0]])
    np.testing.assert_allclose(np.asarray(phys.alpha(below), np.float64), np.asarray(lit.alpha(below), np.float64),
                               rtol=1e-6)
    above = np.array([[0.0, 2.5]])          # under the topography crest, above y = 0
    assert float(np.asarray(lit.alpha(above)).ravel()[0]) < 1e-6 < float(np.asarray(phys.alpha(above)).ravel()[0])
