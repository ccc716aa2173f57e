"""AddressSanitizer + UndefinedBehaviorSanitizer over libwost's host-side C++ (the
segment-tree builder and the sampler / Green's-norm tables) and the C oracle
(sanitizers on host code; GPU sanitizers are not available). The
harness tests/native/sanitize_host.cpp drives ordinary, degenerate and extreme
inputs; any sanitizer finding aborts it (-fno-sanitize-recover)."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
CSRC = os.path.join(REPO, "dcrmontecarlo_amd", "csrc")
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-g", "-O1"]


@pytest.mark.skipif(shutil.which("g++") is None or shutil.which("gcc") is None, reason="needs gcc/g++")
def test_host_code_under_asan_ubsan(tmp_path):
    oracle_o = str(tmp_path / "wost_oracle.o")
    subprocess.run(["gcc", "-std=c11", "-fopenmp", "-ffp-contract=off", *SAN, "-c",
                    os.path.join(REPO, "oracle", "wost_oracle.c"), "-o", oracle_o], check=True)
    exe = str(tmp_path / "sanitize_host")
    subprocess.run(["g++", "-std=c++17", "-fopenmp", *SAN, "-I" + os.path.join(REPO, "include"),
                    os.path.join(HERE, "native", "sanitize_host.cpp"), os.path.join(CSRC, "wost_tree.cpp"),
                    os.path.join(CSRC, "wost_tables.cpp"), oracle_o, "-o", exe, "-lm"], check=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0", UBSAN_OPTIONS="print_stacktrace=1",
               OMP_NUM_THREADS="2")
    r = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "0 failed checks" in r.stdout
