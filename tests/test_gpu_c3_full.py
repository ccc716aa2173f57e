"""C3 at its BASELINE size (BASELINE.json configs[2]: testWostVariableCoefficients,
256 query points x 100k walks, delta tracking with the 32-segment Neumann circle;
bench.py --workload variable_coefficients), through size-independent properties
(the walk-for-walk parity against the reference and the oracle runs at smaller
sizes in tests/test_gpu_parity.py):

* linearity in the source: the walks do not depend on f (solvers/WoStSolver.py:
  242-258), so u(2f) = 2 u(f) bit for bit, and the walk-step counts are equal;
* determinism: the same seed gives the same per-point sums bit for bit;
* block invariance: the solve split into two block ranges (wost_solve) sums to the
  full solve's per-point statistics bit for bit;
* the per-point means agree with the CPU oracle's independent walks (other seed,
  2,048 walks per point) within 4 combined standard errors.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _c3():
    from dcrmontecarlo_amd import scenarios as S

    return S.variable_coefficients(n_points=256, n_walks=100_000)


def test_c3_full_size_linearity_and_determinism(gpu_available):
    from dcrmontecarlo_amd.geometry import PolyLinesSimple
    from dcrmontecarlo_amd.solvers import WostSolver_2D

    sc = _c3()
    assert len(sc.points) == 256
    mk = lambda f: WostSolver_2D(PolyLinesSimple(sc.dirichlet), sc.g, PolyLinesSimple(sc.neumann), source=f,
                                 sigma=sc.sigma, alpha=sc.alpha)
    s1, s2 = mk(sc.f), mk(2.0 * sc.f)
    kw = dict(nWalks=sc.n_walks, maxSteps=sc.max_steps, eps=sc.eps, seed=77, return_stats=True)
    u1, st1 = s1.solve(sc.points, **kw)
    sums1 = s1.last_point_sums.copy()
    assert s1.last_timing["jit"] == 1
    u2, st2 = s2.solve(sc.points, **kw)
    # g vanishes on neither boundary here, so linearity holds for the source part only:
    # u(2f) - u(f) = u_f, with g = 0 in both
    assert st1.total_steps == st2.total_steps > 256 * 100_000
    ug = WostSolver_2D(PolyLinesSimple(sc.dirichlet), 0.0, PolyLinesSimple(sc.neumann), source=sc.f,
                       sigma=sc.sigma, alpha=sc.alpha)
    ug2 = WostSolver_2D(PolyLinesSimple(sc.dirichlet), 0.0, PolyLinesSimple(sc.neumann), source=2.0 * sc.f,
                        sigma=sc.sigma, alpha=sc.alpha)
    _, a = ug.solve(sc.points, **kw)
    _, b = ug2.solve(sc.points, **kw)
    assert np.array_equal(b.mean, 2.0 * a.mean) and a.total_steps == st1.total_steps
    # determinism
    u1b, st1b = s1.solve(sc.points, **kw)
    assert np.array_equal(s1.last_point_sums, sums1) and np.array_equal(st1b.mean, st1.mean)
    # block invariance: two block ranges sum to the full solve's per-point sums
    nb = s1.num_blocks(len(sc.points), sc.n_walks)
    half = nb // 2
    b0 = s1.solve_blocks(sc.points, sc.n_walks, 0, half, sc.max_steps, sc.eps, 77)
    b1 = s1.solve_blocks(sc.points, sc.n_walks, half, nb, sc.max_steps, sc.eps, 77)
    rows = np.concatenate([b0, b1]).reshape(len(sc.points), -1, 3)
    acc = np.zeros((len(sc.points), 3))
    for k in range(rows.shape[1]):
        acc += rows[:, k]
    assert np.array_equal(acc, sums1)


def test_c3_full_size_means_agree_with_the_oracle(gpu_available):
    from oracle import oracle as O

    sc = _c3()
    s = sc.solver(device=0)
    _, st = s.solve(sc.points, nWalks=sc.n_walks, maxSteps=sc.max_steps, eps=sc.eps, seed=5, return_stats=True)
    pts = sc.points[::8]                                   # 32 points along the grid
    W = 2048
    pb = O.Problem.from_scenario(sc, sigma_bar=O.Problem.from_scenario(sc).sigma_bar())
    om, ose, _ = pb.solve(pts, W, sc.max_steps, sc.eps, 99)
    z = (st.mean[::8] - om) / np.sqrt(st.stderr[::8] ** 2 + ose ** 2)
    assert np.all(np.abs(z) < 4.0), z
    assert np.all(st.stderr < 0.02)
