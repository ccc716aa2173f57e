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
HIPRTC_OPTS = ["-O3", "-std=c++17", "-fhip-fp32-correctly-rounded-divide-sqrt", "-ffp-contract=fast-honor-pragmas",
               "-fno-slp-vectorize"]


def test_generated_sources_name_their_variant():
    src = S.dcr_dipole().kernel_source()
    assert "walk kernel, mode 5" in src and "wost_walk_jit" in src
    assert "walk_body<true, true, true, false, false, 1, false, false>" in src
    assert "wost_point_alpha_jit" in src                    # alpha at the query points (delta)
    assert "const float2 v[5]" in src                       # the square compiled in
    # whole-field saturation shortcut of the alpha jet (two smooth circles + a constant)
    assert src.count("wost::sat_sigmoid_radial(x, y, ") == 2 and "if (WOST_SAT_ALL(sat))" in src
    assert "return wost::Jet{alpha(x, y), z, z, z};" in src
    nb = S.notebook_dcr().kernel_source()                   # + sigmoid(10000 y): linear sigmoid predicate
    assert "wost::sat_sigmoid_lin(x, y, " in nb and nb.count("wost::sat_sigmoid_radial(x, y, ") == 2
    vc = S.variable_coefficients().kernel_source()          # detached alpha (Q9): no jet shortcut needed
    assert "if (WOST_SAT_ALL(sat))" not in vc
    # 8+ compiled-in Neumann segments: the two-pass scans (per-vertex line filter, marked
    # silhouettes); C4's single top segment: the unrolled one
    assert "intersect_polylines_lines<33>(v, sN," in vc and "silhouette_distance_compact<33>(v, sN," in vc
    assert "intersect_polylines_lines" not in src and "intersect_polylines<false, 2>(v, 2," in src
    assert "silhouette_distance<2>(v, 2," in src
    topo = S.wenner_topography(n_electrodes=4, n_walks=1).kernel_source()
    assert "walk_body<true, true, true, true, false, 1, false, false>" in topo      # the 10k-segment surface uses the tree
    lap = S.laplace_square().kernel_source()
    assert "walk_body<false, false, false, false, false, 1, false, false>" in lap
    assert "wost_point_alpha_jit" not in lap


def _tabulated_source():
    """A delta-tracking problem whose alpha and source are tabulated (WOST_FK_GRID)."""
    import numpy as np

    from dcrmontecarlo_amd import fields as F
    from dcrmontecarlo_amd.geometry import PolyLinesSimple
    from dcrmontecarlo_amd.solvers.WoStSolver import kernel_source

    sc = S.variable_coefficients()
    xs = np.linspace(-1.6, 1.6, 33, dtype=np.float32)
    a = F.tabulated(1.0 + 0.1 * np.add.outer(xs, xs) ** 2, -1.6, -1.6, 0.1, 0.1)
    f = F.tabulated(np.outer(xs, xs), -1.6, -1.6, 0.1, 0.1) * F.indicator_disk((0, 0), 1.5)
    return kernel_source(PolyLinesSimple(sc.dirichlet), sc.g, PolyLinesSimple(sc.neumann), source=f,
                         sigma=sc.sigma, alpha=a)


def test_tabulated_fields_are_generated():
    src = _tabulated_source()
    assert src.count("wost::fj_grid(grid + ") == 1 and "wost::fv_grid(grid + 0," in src
    assert "reinterpret_cast<const float*>(A.prog + " in src


def _fixed_source(delta=False):
    import numpy as np

    from dcrmontecarlo_amd.fields import X, Y
    from dcrmontecarlo_amd.geometry import PolyLinesSimple
    from dcrmontecarlo_amd.solvers.WoStSolver import kernel_source

    D = PolyLinesSimple(np.array([[0, 1], [0, 0], [1, 0], [1, 1]], np.float32))
    N = PolyLinesSimple(np.array([[1, 1], [0, 1]], np.float32))
    if delta:   # compat="fixed" delta tracking (the corrected screened sampler)
        return kernel_source(D, X, N, source=1.0 + X * Y, sigma=1.0 + Y, alpha=1.0 + 0.5 * X, compat="fixed")
    return kernel_source(D, X, N, source=1.0 + X * Y, compat="fixed")


def test_generated_sources_compile_for_gfx950():
    names = ["laplace_square", "poisson_square", "variable_coefficients", "dcr_dipole", "wenner_topography",
             "tabulated", "fixed_mixed_poisson", "fixed_mixed_delta"]
    with tempfile.TemporaryDirectory() as d:
        procs = []
        for n in names:
            if n == "tabulated":
                src = _tabulated_source()
            elif n == "fixed_mixed_poisson":   # compat="fixed" (wost_walk.h FIX)
                src = _fixed_source()
                assert "walk_body<true, true, false, false, false, 1, true, false>" in src
            elif n == "fixed_mixed_delta":
                src = _fixed_source(delta=True)
                assert "walk_body<true, true, true, false, false, 1, true, false>" in src
            else:
                sc = S.ALL[n]() if n != "wenner_topography" else S.wenner_topography(n_electrodes=4, n_walks=1)
                src = sc.kernel_source()
            path = os.path.join(d, n + ".hip")
            with open(path, "w") as f:
                f.write(src)
            procs.append((n, subprocess.Popen(
                ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "--cuda-device-only", "-c", *HIPRTC_OPTS,
                 "-I" + CSRC, "-I" + os.path.join(REPO, "include"), path, "-o", path + ".o"],
                stdout=subprocess.PIPE, stderr=subprocess.STDOUT)))
        for n, p in procs:
            out = p.communicate(timeout=600)[0].decode()
            assert p.returncode == 0, f"{n}: {out[-2000:]}"
