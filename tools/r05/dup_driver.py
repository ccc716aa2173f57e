"""Round 5: one scenario solve for the phase-duplication PMC passes (tools/r05/phase_dup.sh):
a warm-up solve (JIT), then the measured one; prints its walk-steps and launches.
Usage: dup_driver.py SCENARIO [points] [walks]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
from dcrmontecarlo_amd import scenarios as S  # noqa: E402

SIZES = {"dcr_dipole": (48, 1_000_000), "variable_coefficients": (256, 100_000), "laplace_square": (64, 200_000),
         "poisson_square": (64, 200_000), "wenner_topography": (256, 2000)}


def main():
    name = sys.argv[1]
    n, W = SIZES[name]
    if len(sys.argv) > 2:
        n, W = int(sys.argv[2]), int(sys.argv[3])
    sc = S.ALL[name]()
    s = sc.solver(device=0)
    pts = sc.points[:n]
    s.solve(pts, nWalks=2048, maxSteps=sc.max_steps, eps=sc.eps, seed=1)
    s.solve(pts, nWalks=W, maxSteps=sc.max_steps, eps=sc.eps, seed=7)
    t = s.last_timing
    print(f"dup_driver {name} flags={os.environ.get('WOST_EXP_FLAGS', '0')} steps={t['total_steps']} "
          f"launches={t['n_launches']} kernel_ms={t['walk_kernel_ms']:.3f}", flush=True)


if __name__ == "__main__":
    main()
