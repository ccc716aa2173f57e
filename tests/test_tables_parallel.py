"""The host sampler tables (wost_tables.cpp) are built on up to 8 threads (a fresh
process's first delta-tracking solve waited ~60 ms for the screened sampler's 65,537
density samples on one core): every node and sample is computed by the same code whatever
thread takes it, so the threaded build must write exactly the bytes of the one-thread
build (-DWOST_TABLES_SERIAL) -- Green's and Jacobian nodes, the screened nodes at five
sigma_bar, and compat="fixed"'s 129 x 257 screened table."""
import os
import subprocess

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "dcrmontecarlo_amd", "csrc")


def _dump(tmp_path, serial):
    exe = tmp_path / ("serial" if serial else "threaded")
    cmd = ["g++", "-O2", "-std=c++17", "-pthread", "-I" + CSRC, os.path.join(REPO, "tests", "native", "tables_dump.cpp"),
           os.path.join(CSRC, "wost_tables.cpp"), "-o", str(exe)] + (["-DWOST_TABLES_SERIAL"] if serial else [])
    subprocess.run(cmd, check=True, capture_output=True, timeout=300)
    out = tmp_path / (exe.name + ".bin")
    subprocess.run([str(exe), str(out)], check=True, timeout=300)
    return out.read_bytes()


def test_threaded_tables_equal_one_thread(tmp_path):
    a, b = _dump(tmp_path, True), _dump(tmp_path, False)
    assert len(a) == 4 * (7 * 4097 + 129 * 257)
    assert a == b
