"""Test configuration.

-m "not gpu": the CPU oracle against the reference's golden vectors, the
field DSL, host logic, the C-ABI exports and the multi-rank reduction (gloo).
-m gpu: parity of libwost's HIP kernels with the oracle and the golden vectors.
"""
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); calls libwost kernels")
    config.addinivalue_line("markers", "slow: long-running")


def golden(name):
    path = os.path.join(GOLDEN, name)
    if not os.path.exists(path):
        pytest.skip(f"golden fixture {name} missing (tools/gen_fixtures.py)")
    return np.load(path, allow_pickle=False)


@pytest.fixture(scope="session")
def gpu_available():
    from dcrmontecarlo_amd import _lib
    n = _lib.device_count()
    if n == 0:
        pytest.fail("no HIP device visible: -m gpu tests must run on an MI355X (no CPU fallback exists)")
    return n


@pytest.fixture(autouse=True)
def _compile_before_first_solve(request, monkeypatch):
    """GPU tests check the field-specialised kernels -- and each kernel option -- against the
    oracle, the reference's fixtures and one another, so every solver they build compiles
    its kernel before its first solve (option jit_race = 0). By default (jit_race = 1) a
    solve whose kernel is in no cache runs on the precompiled kernel while it compiles: the
    same bits, tested by tests/test_gpu_race.py, which keeps the default."""
    if request.node.get_closest_marker("gpu") is None or request.node.fspath.basename == "test_gpu_race.py":
        return
    from dcrmontecarlo_amd.solvers import WoStSolver as W

    orig = W.WostSolver_2D.__init__

    def init(self, *a, **k):
        orig(self, *a, **k)
        self.set_option("jit_race", 0)

    monkeypatch.setattr(W.WostSolver_2D, "__init__", init)
