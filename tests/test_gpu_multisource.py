"""Multi-source batching (WostSolver_2D.solve_sources, wost_solve_multi) on the device.

The walks do not depend on the source term (reference solvers/WoStSolver.py:
242-258 draws the same random numbers whatever f is), so scoring S sources
with one set of walks must give, for every source k, exactly the per-walk
values and per-point sums of ``setSourceTerm(sources[k]); solve(...)`` with
the same seed. These tests pin that bit for bit, including the chunking above
WOST_MAX_SOURCES sources, and that the solver's own source is restored.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _solver(name, **kw):
    from dcrmontecarlo_amd import scenarios as S

    sc = S.ALL[name]()
    return sc, sc.solver(**kw)


def _sources(sc, n):
    from dcrmontecarlo_amd import fields as F
    from dcrmontecarlo_amd import survey

    lo = np.asarray(sc.points, np.float64).min(0)
    hi = np.asarray(sc.points, np.float64).max(0)
    out = []
    for k in range(n):
        t = (k + 0.5) / n
        c = lo + t * (hi - lo)
        w = 0.05 * float(np.max(hi - lo) + 1.0)
        out.append(survey.electrode_source(c, w, current=1.0 + k) + 0.25 * k * F.X)
    return out


@pytest.mark.parametrize("param", [0, 1])
@pytest.mark.parametrize("name", ["poisson_square", "dcr_dipole", "variable_coefficients"])
def test_each_source_equals_its_single_source_solve(gpu_available, name, param):
    """param = 1 (option param_sources): the multi-source kernel reads the sources'
    parameters from the program buffer instead of literals -- the same bits."""
    sc, s = _solver(name)
    s.set_option("param_sources", param)
    pts = sc.points[:5]
    W, seed = 3000, 23
    srcs = _sources(sc, 3)
    vals, steps = s.solve_sources_walks(pts, srcs, nWalks=W, maxSteps=sc.max_steps, eps=sc.eps, seed=seed)
    assert vals.shape == (3, len(pts), W) and steps.shape == (len(pts), W)
    u, st = s.solve_sources(pts, srcs, nWalks=W, maxSteps=sc.max_steps, eps=sc.eps, seed=seed, return_stats=True)
    assert u.shape == (3, len(pts))
    for k, f in enumerate(srcs):
        s.setSourceTerm(f)
        v1, s1 = s.solve_walks(pts, nWalks=W, maxSteps=sc.max_steps, eps=sc.eps, seed=seed)
        np.testing.assert_array_equal(steps, s1)
        np.testing.assert_array_equal(vals[k], v1)
        u1, st1 = s.solve(pts, nWalks=W, maxSteps=sc.max_steps, eps=sc.eps, seed=seed, return_stats=True)
        np.testing.assert_array_equal(st.mean[k], st1.mean)
        np.testing.assert_array_equal(st.stderr[k], st1.stderr)
        np.testing.assert_array_equal(u[k], np.asarray(u1).ravel())


def test_more_sources_than_one_launch_and_source_restored(gpu_available):
    from dcrmontecarlo_amd import _lib

    sc, s = _solver("poisson_square")
    pts = sc.points[:3]
    W, seed = 2048, 5
    before = s.solve(pts, nWalks=W, maxSteps=sc.max_steps, eps=sc.eps, seed=seed)
    S = _lib.WOST_MAX_SOURCES + 2
    srcs = _sources(sc, S)
    u = s.solve_sources(pts, srcs, nWalks=W, maxSteps=sc.max_steps, eps=sc.eps, seed=seed)
    assert u.shape == (S, len(pts))
    after = s.solve(pts, nWalks=W, maxSteps=sc.max_steps, eps=sc.eps, seed=seed)
    np.testing.assert_array_equal(np.asarray(before), np.asarray(after))
    for k in (0, _lib.WOST_MAX_SOURCES - 1, S - 1):
        s.setSourceTerm(srcs[k])
        np.testing.assert_array_equal(u[k], np.asarray(s.solve(pts, nWalks=W, maxSteps=sc.max_steps, eps=sc.eps,
                                                               seed=seed)).ravel())


def test_single_source_list_and_none_entries(gpu_available):
    sc, s = _solver("poisson_square")
    pts = sc.points[:2]
    u = s.solve_sources(pts, [sc.f, None], nWalks=1024, maxSteps=sc.max_steps, eps=sc.eps, seed=1)
    base = np.asarray(s.solve(pts, nWalks=1024, maxSteps=sc.max_steps, eps=sc.eps, seed=1)).ravel()
    np.testing.assert_array_equal(u[0], base)
    s.setSourceTerm(0.0)
    np.testing.assert_array_equal(u[1], np.asarray(s.solve(pts, nWalks=1024, maxSteps=sc.max_steps, eps=sc.eps,
                                                           seed=1)).ravel())


def test_api_errors(gpu_available):
    sc, s = _solver("poisson_square")
    with pytest.raises(ValueError):
        s.solve_sources(sc.points[:2], [], nWalks=16)
    s.set_jit(False)
    with pytest.raises(NotImplementedError):
        s.solve_sources(sc.points[:2], _sources(sc, 2), nWalks=16)
    # a one-source list still runs on the precompiled kernel
    s.solve_sources(sc.points[:2], _sources(sc, 1), nWalks=16)


def test_homogeneous_survey_apparent_resistivity_is_background(gpu_available):
    """Model == background: every quadripole's rho_a is 1/alpha_bg
    (the two solves share walks and sources, so dV_model == dV_background bit for bit)."""
    from dcrmontecarlo_amd import scenarios as S
    from dcrmontecarlo_amd import survey

    sc = S.dcr_dipole(n_electrodes=8, n_walks=2000)
    sc_h = survey.homogeneous(sc, 0.01)
    r = survey.run_dipole_dipole_survey(sc_h, 0.01, n_walks=2000, n_max=2, width=0.5, seed=3)
    assert r.quadripoles.shape[0] == len(survey.dipole_dipole_quadripoles(8, 2))
    assert r.u_model.shape == (len(r.transmitters), 8)
    np.testing.assert_array_equal(r.model.dv, r.background.dv)
    ok = r.background.dv != 0
    assert ok.all()
    np.testing.assert_allclose(r.rho.rho_a[ok], 100.0, rtol=1e-12)


@pytest.mark.parametrize("name", ["dcr_dipole", "wenner_topography"])
def test_prepared_kernel_is_the_one_the_solve_launches(gpu_available, name):
    """wost_prepare_sources (survey.prepare_survey_kernels): preparing a group's kernel
    from several threads at once -- also on one handle -- compiles exactly the kernel its
    solve_sources then looks up (no compile in the solve: jit_ms == 0), and the solve's
    bits equal those of an unprepared handle's."""
    import threading

    from dcrmontecarlo_amd import scenarios as S

    sc = S.ALL[name](**({"n_electrodes": 32, "n_walks": 256} if name == "wenner_topography" else {}))
    pts = sc.points[:6]
    W, seed = 1024, 31
    # sources no other test compiled: a fresh kernel for this process's module cache
    rng = np.random.default_rng()
    srcs = _sources(sc, 4)
    srcs = [f * float(1.0 + rng.uniform(0.01, 0.02)) for f in srcs]
    prepared = sc.solver()
    errs = []

    def prep():
        try:
            prepared.prepare_sources(srcs, len(pts))
        except Exception as e:  # noqa: BLE001
            errs.append(e)

    th = [threading.Thread(target=prep) for _ in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs
    u, st = prepared.solve_sources(pts, srcs, nWalks=W, maxSteps=sc.max_steps, eps=sc.eps, seed=seed,
                                   return_stats=True)
    assert prepared.last_timing["jit_ms"] == 0.0
    other = sc.solver()
    u2, st2 = other.solve_sources(pts, srcs, nWalks=W, maxSteps=sc.max_steps, eps=sc.eps, seed=seed,
                                  return_stats=True)
    np.testing.assert_array_equal(np.asarray(u), np.asarray(u2))
    np.testing.assert_array_equal(st.stderr, st2.stderr)


def test_prepare_sources_argument_errors(gpu_available):
    sc, s = _solver("poisson_square")
    with pytest.raises(Exception):
        s.prepare_sources(_sources(sc, 2), 0)
    s.set_jit(False)
    with pytest.raises(Exception):
        s.prepare_sources(_sources(sc, 2), 4)
