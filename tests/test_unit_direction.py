"""The walk's ray-direction normalisation (wost_device.h unit_direction) is
bit for bit sqrtf and IEEE division (PolylinesSimple.py:151-152): closed-form
square roots and reciprocals for the 129 values s2 = |d|^2 within 64 ulps of 1,
and the Markstein division for every float mantissa against each of them."""
import ctypes
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


def test_unit_direction_is_ieee_exact(tmp_path):
    out = str(tmp_path / "libunit_dir_check.so")
    # host build of the __host__ __device__ header; -ffp-contract=off like the kernels' geometry
    subprocess.run(["/opt/rocm/bin/hipcc", "-O2", "-std=c++17", "-fPIC", "-shared", "--offload-arch=gfx950",
                    "-ffp-contract=off", "-I" + os.path.join(REPO, "include"), "-x", "hip",
                    os.path.join(HERE, "native", "unit_dir_check.cpp"), "-o", out], check=True)
    lib = ctypes.CDLL(out)
    c = (ctypes.c_long * 5)()
    assert lib.unit_dir_check(c) == 0
    bad_sqrt, bad_rcp, bad_div, n_div, bad_fn = list(c)
    assert n_div == 65 * (1 << 23)
    assert (bad_sqrt, bad_rcp, bad_div, bad_fn) == (0, 0, 0, 0)
