"""The hiprtc kernel generator (wost_jit.cpp), checked on the build machine:
wost_kernel_source() returns, without a device, the source wost_create would
compile; it must compile for gfx950 with the options libwost gives hiprtc
(wost_jit.cpp, compile()), for every kernel variant the scenarios use."""
import os
import subprocess
import tempfile

import pytest

from dcrmontecarlo_amd import scenarios as S

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "dcrmontecarlo_amd", "csrc")
HIPRTC_OPTS = ["-O3", "-std=c++17", "-fhip-fp32-correctly-rounded-divide-sqrt", "-ffp-contract=fast-honor-pragmas"]


def test_generated_sources_name_their_variant():
    src = S.dcr_dipole().kernel_source()
    assert "walk kernel, mode 5" in src and "wost_walk_jit" in src
    assert "walk_body<true, true, true, false, false>" in src
    assert "const float2 v[5]" in src                       # the square compiled in
    topo = S.wenner_topography(n_electrodes=4, n_walks=1).kernel_source()
    assert "walk_body<true, true, true, true, false>" in topo      # the 10k-segment surface uses the tree
    lap = S.laplace_square().kernel_source()
    assert "walk_body<false, false, false, false, false>" in lap


def test_generated_sources_compile_for_gfx950():
    names = ["laplace_square", "poisson_square", "variable_coefficients", "dcr_dipole", "wenner_topography"]
    with tempfile.TemporaryDirectory() as d:
        procs = []
        for n in names:
            sc = S.ALL[n]() if n != "wenner_topography" else S.wenner_topography(n_electrodes=4, n_walks=1)
            path = os.path.join(d, n + ".hip")
            with open(path, "w") as f:
                f.write(sc.kernel_source())
            procs.append((n, subprocess.Popen(
                ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "--cuda-device-only", "-c", *HIPRTC_OPTS,
                 "-I" + CSRC, "-I" + os.path.join(REPO, "include"), path, "-o", path + ".o"],
                stdout=subprocess.PIPE, stderr=subprocess.STDOUT)))
        for n, p in procs:
            out = p.communicate(timeout=600)[0].decode()
            assert p.returncode == 0, f"{n}: {out[-2000:]}"
