"""The walk kernels draw philox4x32_10({k, 0, g_lo, g_hi}) with rounds 0 and 1's
per-walk work hoisted to the walk's refill (wost_device.h philox_walk /
philox_draw): bit for bit the full bijection, checked on the host build of the
header over 200k random walk ids, keys and steps (the full bijection itself is
pinned to Random123 / rocRAND in tests/test_oracle_golden.py)."""
import ctypes
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


def test_split_philox_is_philox4x32_10(tmp_path):
    out = str(tmp_path / "libphilox_check.so")
    subprocess.run(["/opt/rocm/bin/hipcc", "-O2", "-std=c++17", "-fPIC", "-shared", "--offload-arch=gfx950",
                    "-I" + os.path.join(REPO, "include"), "-x", "hip", os.path.join(HERE, "native", "philox_check.cpp"),
                    "-o", out], check=True)
    lib = ctypes.CDLL(out)
    lib.philox_split_check.restype = ctypes.c_long
    assert lib.philox_split_check(ctypes.c_long(200_000)) == 0
