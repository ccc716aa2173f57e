"""The communicator's id exchange under the real launcher: torchrun (static
rendezvous, its elastic agent hosting the TCP store on MASTER_PORT) starts two CPU
processes that run comm.exchange_over_store; both must read rank 0's bytes. This
is the bootstrap bench.py uses for N > 1 (Communicator.from_env); the RCCL part
needs GPUs and is covered on the device by tests/test_gpu_distributed.py."""
import os
import socket
import subprocess
import sys
import textwrap

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_id_exchange_under_torchrun(tmp_path):
    script = tmp_path / "worker.py"
    script.write_text(textwrap.dedent(f"""
        import os, sys
        sys.path.insert(0, {REPO!r})
        from dcrmontecarlo_amd import comm
        rank = int(os.environ["RANK"])
        uid, store = comm.exchange_over_store(lambda: bytes(range(128)) if rank == 0 else b"wrong", timeout=60)
        assert uid == bytes(range(128)), uid[:8]
        store.set("done%d" % rank, b"1")
        for r in range(int(os.environ["WORLD_SIZE"])):
            store.get("done%d" % r)
        print("rank", rank, "ok", flush=True)
    """))
    port = _free_port()
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), str(script)],
                       capture_output=True, text=True, timeout=240, env=dict(os.environ, OMP_NUM_THREADS="1"))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    assert r.stdout.count(" ok") == 2


def test_store_binds_every_interface_for_a_multinode_loopback_master(monkeypatch):
    """a multi-node job whose MASTER_ADDR resolves to loopback on rank 0's node
    listens on every interface; a single-node job on MASTER_ADDR itself; WOST_STORE_BIND wins."""
    from dcrmontecarlo_amd import comm

    monkeypatch.delenv("WOST_STORE_BIND", raising=False)
    monkeypatch.setenv("WORLD_SIZE", "16")
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "8")
    assert comm._bind_address("127.0.0.1") == ""
    assert comm._bind_address("localhost") == ""
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "16")
    assert comm._bind_address("127.0.0.1") == "127.0.0.1"
    monkeypatch.setenv("WOST_STORE_BIND", "0.0.0.0")
    assert comm._bind_address("127.0.0.1") == "0.0.0.0"


def test_process_start_time_without_psutil(monkeypatch):
    """without psutil the start comes from /proc (not "now", which made a late
    rank ignore a valid id file); the file store then accepts a file written just before."""
    import builtins
    import time

    from dcrmontecarlo_amd import comm

    real = builtins.__import__

    def no_psutil(name, *a, **kw):
        if name == "psutil":
            raise ImportError("no psutil")
        return real(name, *a, **kw)

    monkeypatch.setattr(builtins, "__import__", no_psutil)
    t = comm._process_start_time()
    assert t is not None and t <= time.time() + 1.0 and t > time.time() - 86400 * 365
