"""The out-of-process compile helper (dcrmontecarlo_amd/wost_jitc, wost_jit.cpp
compile_in_helper), on the build machine without a device: wost_jit_compile through the
helper returns the same code object bytes as hiprtc in this process, for a single-source
kernel (C4) and a multi-source survey kernel (C5); a source that does not compile fails
with the compiler's message; and compiles of concurrent threads overlap in helpers where
in-process compiles wait for one another (ROCm's compiler library serialises one
process's compiles: the C5 survey's cold start)."""
import ctypes
import os
import subprocess
import sys
import threading
import time

import pytest

from dcrmontecarlo_amd import _lib
from dcrmontecarlo_amd import scenarios as S

HELPER = os.path.join(os.path.dirname(_lib.LIB_PATH), "wost_jitc")


@pytest.fixture(autouse=True)
def _private_comgr_cache(tmp_path, monkeypatch):
    # comgr caches hiprtc's compiles on disk: a private cache per test, so that the
    # compiles here really run (and the helper children inherit it)
    monkeypatch.setenv("AMD_COMGR_CACHE_DIR", str(tmp_path / "comgr"))


def compile_source(src: str, in_process: bool):
    n, used = ctypes.c_int64(), ctypes.c_int32(-1)
    buf = (ctypes.c_uint8 * (8 << 20))()
    rc = _lib.lib.wost_jit_compile(src.encode(), b"gfx950", 1 if in_process else 0, buf, len(buf), ctypes.byref(n),
                                   ctypes.byref(used))
    return rc, bytes(buf[:n.value]) if rc == 0 else b"", used.value


def _survey_source(g=3):
    from dcrmontecarlo_amd import survey as SV

    sc = S.wenner_topography(n_walks=1)
    srcs = [SV.dipole_source(sc.points[q], sc.points[q + 3], 0.5) for q in range(len(sc.points) - 3)]
    j0, j1, t0, t1 = list(SV.wenner_batches(len(sc.points)))[g]
    return sc.kernel_source(sources=srcs[t0:t1])


def test_helper_is_installed_next_to_the_library():
    assert os.access(HELPER, os.X_OK), "make -C dcrmontecarlo_amd/csrc builds wost_jitc next to libwost.so"


EQUAL = r"""
import sys
sys.path.insert(0, %r)
sys.path.insert(0, %r)
import test_jit_helper as T
from dcrmontecarlo_amd import scenarios as S
src = S.dcr_dipole().kernel_source() if sys.argv[1] == "dcr_dipole" else T._survey_source()
rc_h, code_h, used_h = T.compile_source(src, in_process=False)
rc_i, code_i, used_i = T.compile_source(src, in_process=True)
assert rc_h == 0 and rc_i == 0
assert used_h == 1 and used_i == 0
assert len(code_h) > 1000 and code_h[:4] == b"\x7fELF"
print("equal" if code_h == code_i else "differ", len(code_h), len(code_i))
"""


@pytest.mark.parametrize("which", ["dcr_dipole", "wenner_survey_group"])
def test_helper_code_object_equals_in_process(which, tmp_path):
    # in a fresh process that has not imported PyTorch: libwost then binds /opt/rocm's
    # hiprtc, the helper's compiler (PyTorch-ROCm's own copy is another ROCm release's,
    # which the kernel cache key tells apart: wost_jit.cpp cache_identity)
    here = os.path.dirname(os.path.abspath(__file__))
    env = dict(os.environ, AMD_COMGR_CACHE_DIR=str(tmp_path / "comgr"))
    out = subprocess.run([sys.executable, "-c", EQUAL % (os.path.dirname(here), here), which], env=env,
                         capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-3000:]
    assert out.stdout.split()[0] == "equal", out.stdout


def test_a_source_that_does_not_compile_reports_the_compiler():
    rc, _, _ = compile_source('#include "wost_walk.h"\nthis is not C++;\n', in_process=False)
    assert rc == _lib.WOST_ERR_UNSUPPORTED
    assert "hiprtc" in _lib.lib.wost_last_error().decode()


def test_capacity_and_arguments():
    src = S.laplace_square().kernel_source().encode()
    n = ctypes.c_int64()
    assert _lib.lib.wost_jit_compile(src, b"gfx950", 0, None, 0, ctypes.byref(n), None) == 0 and n.value > 1000
    small = (ctypes.c_uint8 * 16)()
    assert _lib.lib.wost_jit_compile(src, b"gfx950", 0, small, 16, ctypes.byref(n), None) == _lib.WOST_ERR_INVALID_ARG
    assert _lib.lib.wost_jit_compile(None, b"gfx950", 0, None, 0, ctypes.byref(n), None) == _lib.WOST_ERR_INVALID_ARG
    assert _lib.lib.wost_jit_compile(src, b"", 0, None, 0, ctypes.byref(n), None) == _lib.WOST_ERR_INVALID_ARG


def test_jit_process_is_a_launch_option():
    # it selects where the compile runs, never the code: not reported as a kernel change
    assert _lib.options_report()["non_default"] == {}


def test_concurrent_compiles_overlap_in_helpers():
    srcs = [_survey_source(g) for g in range(4)]

    def wall(in_process):
        errs = []
        th = [threading.Thread(target=lambda s=s: errs.append(compile_source(s, in_process)[0])) for s in srcs]
        t0 = time.perf_counter()
        for t in th:
            t.start()
        for t in th:
            t.join()
        assert errs == [0] * len(srcs)
        return time.perf_counter() - t0

    helper = wall(False)
    os.environ["AMD_COMGR_CACHE_DIR"] += "_2"   # (monkeypatch restores it)
    in_process = wall(True)
    # four compiles: in-process they run one after another, in helpers at once (the
    # container has >= 4 cores); a loose bound keeps a loaded machine from failing it
    assert helper < 0.6 * in_process, (helper, in_process)
