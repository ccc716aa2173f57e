"""bench.py's own multi-rank launch (no GPU): ``--gpus N`` without a launcher starts N
rank processes with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, from a parent that
imports nothing of the package (no HIP call), and returns non-zero when a rank fails,
after stopping the others. Under a launcher, --gpus must equal WORLD_SIZE."""
import json
import os
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
BENCH = os.path.join(REPO, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    env.update(kw)
    return env


def test_dry_launch_starts_every_rank():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "3", "--dry-launch"], capture_output=True, text=True,
                       timeout=120, env=_env())
    assert r.returncode == 0, r.stderr[-2000:]
    ranks = [json.loads(line) for line in r.stdout.splitlines() if line.startswith("{")]
    assert sorted(x["rank"] for x in ranks) == [0, 1, 2]
    assert all(x["local_rank"] == x["rank"] and x["world_size"] == 3 for x in ranks)
    assert len({x["master_port"] for x in ranks}) == 1 and ranks[0]["master_addr"] == "127.0.0.1"
    assert len({x["ppid"] for x in ranks}) == 1          # children of one launcher process
    assert len({x["pid"] for x in ranks}) == 3


def test_dry_launch_propagates_a_rank_failure_and_stops_the_others():
    t0 = time.time()
    r = subprocess.run([sys.executable, BENCH, "--gpus", "3", "--dry-launch", "--dry-launch-fail-rank", "1"],
                       capture_output=True, text=True, timeout=120, env=_env())
    assert r.returncode == 3, (r.returncode, r.stderr[-2000:])
    assert "rank 1 exited with status 3" in r.stderr
    assert time.time() - t0 < 25            # the healthy ranks (sleeping 30 s) were stopped


def test_gpus_must_match_the_launchers_world_size():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dry-launch"], capture_output=True, text=True,
                       timeout=120, env=_env(WORLD_SIZE="4", RANK="0", LOCAL_RANK="0"))
    assert r.returncode != 0 and "WORLD_SIZE=4" in r.stderr
    r = subprocess.run([sys.executable, BENCH, "--gpus", "4", "--dry-launch"], capture_output=True, text=True,
                       timeout=120, env=_env(WORLD_SIZE="4", RANK="2", LOCAL_RANK="2"))
    assert r.returncode == 0 and json.loads(r.stdout)["rank"] == 2


def test_launch_parent_never_imports_the_package():
    """The launcher parent's import list: numpy and the standard library, nothing that
    initialises HIP (the package, torch)."""
    code = ("import runpy, sys; sys.argv = ['bench.py', '--gpus', '2', '--dry-launch']\n"
            "try:\n    runpy.run_path(%r, run_name='__main__')\nexcept SystemExit as e:\n    rc = e.code\n"
            "bad = [m for m in sys.modules if m.startswith(('dcrmontecarlo_amd', 'torch', 'oracle'))]\n"
            "print('IMPORTED', bad, 'RC', rc)\n") % BENCH
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120, env=_env())
    assert "IMPORTED [] RC 0" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]
