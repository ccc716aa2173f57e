"""wost_set_option / wost_options_report (include/wost.h) and the product library's
environment: libwost.so reads no variable that changes a kernel or a result
(VERDICT r05 Weak #3). The A/B knobs and the result-changing ablations exist only in the
study build (make -C dcrmontecarlo_amd/csrc study -> build/libwost_study.so), which the
tools point WOST_LIB at; bench.py refuses to report a metric from it."""
import json
import os
import subprocess
import sys

import pytest

from dcrmontecarlo_amd import _lib

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STUDY_LIB = os.path.join(REPO, "build", "libwost_study.so")

# every A/B or ablation variable the tools ever set (tools/*.sh, profiles/), and the old
# handle defaults
AB_ENV = {"WOST_EXP_FLAGS": "32", "WOST_JIT": "0", "WOST_TRIG": "fast", "WOST_TREE_LEAF": "3",
          "WOST_TREE_MIN_SEGMENTS": "-1", "WOST_JIT_WAVES": "3", "WOST_JIT_CONST_VERTICES": "0",
          "WOST_JIT_PHILOX_AHEAD": "2", "WOST_JIT_REFILL_MIN": "9", "WOST_JIT_TREE_SHARE": "0",
          "WOST_JIT_SLP": "1", "WOST_JIT_SCHED": "max-ilp", "WOST_TREE_ITER_STATS": "1",
          "WOST_KERNEL_SOURCE_STAGE": "2", "WOST_POOL_SLOTS": "2", "WOST_CHUNK0": "3"}

SOURCE = r"""
import json, sys
sys.path.insert(0, %r)
from dcrmontecarlo_amd import _lib, scenarios as S
out = {"report": _lib.options_report()}
for name in ("dcr_dipole", "wenner_topography", "variable_coefficients"):
    kw = {"n_walks": 1} if name != "variable_coefficients" else {}
    out[name] = S.ALL[name](**kw).kernel_source()
print(json.dumps(out))
"""


def _sources(env_extra, lib=None):
    env = {k: v for k, v in os.environ.items() if not k.startswith("WOST_")}
    env.update(env_extra)
    if lib:
        env["WOST_LIB"] = lib
    r = subprocess.run([sys.executable, "-c", SOURCE % REPO], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_product_library_ignores_the_ab_environment():
    """The generated kernels (the host-only wost_kernel_source) are the same bytes with
    and without every A/B variable set, and the library reports itself as the product."""
    base = _sources({})
    ab = _sources(AB_ENV)
    assert base["report"] == {"build": "product", "non_default": {}}
    assert ab["report"] == base["report"]
    for name in ("dcr_dipole", "wenner_topography", "variable_coefficients"):
        assert ab[name] == base[name], name
    assert "WOST_ABL_NO_RAY" not in ab["dcr_dipole"]


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc"), reason="needs hipcc")
def test_study_library_reads_the_ablations():
    """The same variable changes the study build's kernel: the test above has power."""
    r = subprocess.run(["make", "-s", "-C", os.path.join(REPO, "dcrmontecarlo_amd", "csrc"), "-j8", "study"],
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-2000:]
    base = _sources({}, STUDY_LIB)
    ab = _sources({"WOST_EXP_FLAGS": "32"}, STUDY_LIB)
    assert base["report"]["build"] == "study" and base["report"]["non_default"] == {}
    assert ab["report"]["non_default"] == {"exp_flags": 32}
    assert "WOST_ABL_NO_RAY" in ab["dcr_dipole"] and "WOST_ABL_NO_RAY" not in base["dcr_dipole"]


def test_options_report_without_a_handle():
    assert _lib.options_report() == {"build": "product", "non_default": {}}


def test_bench_refuses_a_study_library():
    """bench.py exits non-zero (and prints no metric line) when its library is a study
    build or a handle option is not the default."""
    if not os.path.exists(STUDY_LIB):
        pytest.skip("no study build")
    env = {k: v for k, v in os.environ.items() if not k.startswith("WOST_")}
    env["WOST_LIB"] = STUDY_LIB
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--steps", "1", "--warmup", "0"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert '"metric"' not in r.stdout
    assert "study build" in r.stderr
