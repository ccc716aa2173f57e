"""A solve whose field-specialised kernel is in no cache (option jit_race, wost_api.hip
solve_race): the kernel compiles in a helper process while the precompiled kernel runs the
walks in ranges of every point, and the specialised kernel takes over the rest once it is
ready. Each walk's value and step count depend only on (seed, walk id), and the two
kernels compute every walk bit for bit alike (test_jit_kernel_matches_interpreted_kernel),
so the raced solve must equal a warm solve on the specialised kernel bit for bit: point
sums, block order, per-walk values and step counts. The reference calls solve() once per
script (tests/testWostWithSource.py:110): this is the solve its users run.

Each test perturbs a field by a random factor so that its kernel is new to this process
(the in-memory module cache) and to the disk cache."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _fresh(name, rng, **kw):
    """A scenario whose source (or boundary values) carries a random factor: a kernel no
    other solve of this process compiled."""
    from dcrmontecarlo_amd import scenarios as S

    sc = S.ALL[name](**kw)
    k = float(1.0 + rng.uniform(1e-3, 2e-3))
    if sc.f is not None:
        sc.f = sc.f * k
    else:
        sc.g = sc.g * k
    return sc


def _warm(sc):
    s = sc.solver()
    s.set_option("jit_race", 0)
    return s


@pytest.mark.parametrize("name,n,W", [("poisson_square", 16, 10_000), ("laplace_square", 16, 3000),
                                      ("variable_coefficients", 32, 20_000), ("dcr_dipole", 12, 40_000),
                                      ("wenner_topography", 64, 512)])
def test_raced_first_solve_equals_the_specialised_kernel(gpu_available, name, n, W):
    rng = np.random.default_rng()
    kw = {"n_electrodes": 64, "n_walks": W} if name == "wenner_topography" else {}
    sc = _fresh(name, rng, **kw)
    pts = sc.points[:n]
    cold = sc.solver()
    u0, st0 = cold.solve(pts, nWalks=W, maxSteps=sc.max_steps, eps=sc.eps, seed=17, return_stats=True)
    t0 = cold.last_timing
    assert t0["precompiled_walks"] > 0, "the first solve did not start on the precompiled kernel"
    assert t0["jit_ms"] == 0.0                      # it did not wait for the compile
    warm = _warm(sc)
    u1, st1 = warm.solve(pts, nWalks=W, maxSteps=sc.max_steps, eps=sc.eps, seed=17, return_stats=True)
    assert warm.last_timing["jit"] == 1 and warm.last_timing["precompiled_walks"] == 0
    np.testing.assert_array_equal(np.asarray(u0), np.asarray(u1))
    np.testing.assert_array_equal(st0.stderr, st1.stderr)
    np.testing.assert_array_equal(st0.mean_steps, st1.mean_steps)
    assert st0.total_steps == st1.total_steps
    # the second solve on the raced handle: the specialised kernel (it waited for the compile
    # if that was still running), the same bits
    u2 = cold.solve(pts, nWalks=W, maxSteps=sc.max_steps, eps=sc.eps, seed=17)
    assert cold.last_timing["jit"] == 1 and cold.last_timing["precompiled_walks"] == 0
    np.testing.assert_array_equal(np.asarray(u2), np.asarray(u1))


def test_raced_per_walk_outputs(gpu_available):
    """solve_walks through the race: every walk's value and step count in its slot."""
    rng = np.random.default_rng()
    sc = _fresh("dcr_dipole", rng)
    pts = sc.points[20:26]
    W = 9000   # (not a whole number of 4096-walk blocks)
    cold = sc.solver()
    v0, s0 = cold.solve_walks(pts, nWalks=W, maxSteps=sc.max_steps, eps=sc.eps, seed=5)
    assert cold.last_timing["precompiled_walks"] > 0
    v1, s1 = _warm(sc).solve_walks(pts, nWalks=W, maxSteps=sc.max_steps, eps=sc.eps, seed=5)
    np.testing.assert_array_equal(s0, s1)
    np.testing.assert_array_equal(v0.view(np.uint32), v1.view(np.uint32))


def test_raced_solve_switches_to_the_specialised_kernel(gpu_available):
    """A solve long enough to outlast the compile (C4's 48 electrodes x 16M walks: ~2.6 s on
    the precompiled kernel, a compile takes ~0.3 s): the precompiled kernel runs its first
    ranges, the specialised one the rest, and the point sums are those of one warm solve."""
    rng = np.random.default_rng()
    sc = _fresh("dcr_dipole", rng)
    W = 16 << 20
    cold = sc.solver()
    u0, st0 = cold.solve(sc.points, nWalks=W, maxSteps=sc.max_steps, eps=sc.eps, seed=3, return_stats=True)
    t0 = cold.last_timing
    total = len(sc.points) * W
    print("raced:", t0["precompiled_walks"], "of", total, "walks on the precompiled kernel;", t0["n_launches"],
          "launches")
    assert 0 < t0["precompiled_walks"] < total and t0["jit"] == 1
    u1, st1 = _warm(sc).solve(sc.points, nWalks=W, maxSteps=sc.max_steps, eps=sc.eps, seed=3, return_stats=True)
    np.testing.assert_array_equal(np.asarray(u0), np.asarray(u1))
    np.testing.assert_array_equal(st0.stderr, st1.stderr)
    assert st0.total_steps == st1.total_steps


def test_no_race_when_the_kernel_is_cached(gpu_available):
    """A fresh handle whose kernel this process already compiled: no precompiled walks."""
    from dcrmontecarlo_amd import scenarios as S

    sc = S.poisson_square()
    a = sc.solver()
    a.solve(sc.points[:4], nWalks=4096, maxSteps=sc.max_steps, eps=sc.eps, seed=1)
    a.solve(sc.points[:4], nWalks=4096, maxSteps=sc.max_steps, eps=sc.eps, seed=1)   # (compiled by now)
    b = sc.solver()
    b.solve(sc.points[:4], nWalks=4096, maxSteps=sc.max_steps, eps=sc.eps, seed=1)
    assert b.last_timing["precompiled_walks"] == 0 and b.last_timing["jit"] == 1


@pytest.mark.parametrize("case", ["fixed_poisson", "long_dirichlet"])
def test_raced_solve_other_kernel_shapes(gpu_available, case):
    """The race under compat="fixed" (the corrected estimator's kernels) and with a
    Dirichlet polyline too long to stage (the specialised kernel reads it from global
    memory, the precompiled one stages it): the same bits as a warm specialised solve."""
    from dcrmontecarlo_amd.fields import X, Y
    from dcrmontecarlo_amd.geometry import PolyLinesSimple
    from dcrmontecarlo_amd.solvers import WostSolver_2D

    k = float(1.0 + np.random.default_rng().uniform(1e-3, 2e-3))   # a kernel new to this process
    if case == "fixed_poisson":
        D = np.array([[-1, -1], [1, -1], [1, 1], [-1, 1], [-1, -1]], np.float32)
        mk = lambda: WostSolver_2D(PolyLinesSimple(D), X**3 + Y**2, source=(-6.0 * X - 2.0) * k, compat="fixed")
        pts = np.array([[0.1, 0.2], [-0.4, 0.5], [0.7, -0.6]], np.float32)
    else:
        t = np.linspace(0.0, 2.0 * np.pi, 6001, dtype=np.float64)
        D = np.stack([np.cos(t), np.sin(t)], axis=1).astype(np.float32)
        D[-1] = D[0]
        mk = lambda: WostSolver_2D(PolyLinesSimple(D), (X**2 - Y**2) * k)
        pts = np.array([[0.1, 0.2], [-0.5, 0.3], [0.0, -0.7]], np.float32)
    cold = mk()
    v0, s0 = cold.solve_walks(pts, nWalks=6000, maxSteps=1000, eps=1e-3, seed=9)
    assert cold.last_timing["precompiled_walks"] > 0
    warm = mk()
    warm.set_option("jit_race", 0)
    v1, s1 = warm.solve_walks(pts, nWalks=6000, maxSteps=1000, eps=1e-3, seed=9)
    assert warm.last_timing["jit"] == 1
    np.testing.assert_array_equal(s0, s1)
    np.testing.assert_array_equal(v0.view(np.uint32), v1.view(np.uint32))


def test_raced_solve_in_ragged_ranges(gpu_available):
    """Several precompiled ranges and a last range that ends inside a 4096-walk block
    (48 electrodes x 100,001 walks: the first range is 12,288 walks of every electrode):
    block sums, their order and the per-walk outputs are one launch's."""
    rng = np.random.default_rng()
    sc = _fresh("dcr_dipole", rng)
    W = 100_001
    cold = sc.solver()
    v0, s0 = cold.solve_walks(sc.points, nWalks=W, maxSteps=sc.max_steps, eps=sc.eps, seed=21)
    t0 = cold.last_timing
    assert t0["precompiled_walks"] > 0 and t0["n_launches"] >= 2, t0
    warm = _warm(sc)
    v1, s1 = warm.solve_walks(sc.points, nWalks=W, maxSteps=sc.max_steps, eps=sc.eps, seed=21)
    np.testing.assert_array_equal(s0, s1)
    np.testing.assert_array_equal(v0.view(np.uint32), v1.view(np.uint32))
    u0, st0 = sc.solver().solve(sc.points, nWalks=W, maxSteps=sc.max_steps, eps=sc.eps, seed=21, return_stats=True)
    u1, st1 = warm.solve(sc.points, nWalks=W, maxSteps=sc.max_steps, eps=sc.eps, seed=21, return_stats=True)
    np.testing.assert_array_equal(np.asarray(u0), np.asarray(u1))
    np.testing.assert_array_equal(st0.stderr, st1.stderr)
