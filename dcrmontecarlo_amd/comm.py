"""Multi-GPU solves through libwost's own RCCL communicator (include/wost.h, "Multi-GPU").

One process per GPU. Rank r solves the walk range ``shard_walk_range(W, R, r)`` of
EVERY point (whole blocks of WOST_BLOCK_WALKS walks, about W / R walks of each point,
so ranks stay balanced whatever the points' walk lengths), the per-block partial sums
are all-gathered over RCCL (xGMI on MI355X), and every rank sums them per point in
global block order: the result is bitwise that of a one-GPU solve for any R
(SURVEY.md 8e). The reference has no parallel code.

The only thing libwost needs from outside is the 128-byte RCCL unique id, made on one
rank and handed to the others. ``Communicator.from_env`` does it without PyTorch: rank 0
hosts a small key-value store on MASTER_ADDR:MASTER_PORT (:class:`SocketStore`, the
standard library's sockets); under torchrun, whose elastic agent already listens on
MASTER_PORT, the ranks of one node meet in a file named after the launch's own values
(MASTER_ADDR, MASTER_PORT, TORCHELASTIC_RUN_ID, restart count) instead, and only a
multi-node torchrun job uses torch's TCPStore client.
``from_torch`` takes an initialised torch.distributed group, ``from_file`` a file every
rank can read.
"""
from __future__ import annotations

import ctypes
import ipaddress
import os
import socket
import socketserver
import struct
import tempfile
import threading
import time

import numpy as np

from . import _lib


_MAX_KEY, _MAX_VALUE = 1024, 4096      # the store carries ids (128 B) and short flags


class _StoreHandler(socketserver.StreamRequestHandler):
    """One client connection: requests b"S" key value (set) and b"G" key (get, waits
    until the key is set); keys and values are length-prefixed (u32, big endian), keys
    at most 1 KiB and values 4 KiB (a longer prefix ends the connection). A key is set
    once: a second b"S" of it is refused (b"\x01"), so no peer can replace an id that
    rank 0 published."""

    def _read(self, cap):
        n = struct.unpack(">I", self.rfile.read(4))[0]
        if n > cap:
            raise OSError(f"store: field of {n} bytes exceeds {cap}")
        return self.rfile.read(n)

    def handle(self):
        try:
            self._serve()
        except (OSError, struct.error):   # a client that went away mid-request
            return

    def _serve(self):
        st = self.server.store
        while True:
            op = self.rfile.read(1)
            if not op:
                return
            key = self._read(_MAX_KEY)
            if op == b"S":
                val = self._read(_MAX_VALUE)
                with st.cond:
                    fresh = key not in st.kv
                    if fresh:
                        st.kv[key] = val
                        st.cond.notify_all()
                self.wfile.write(b"\x00" if fresh else b"\x01")
            elif op == b"G":
                with st.cond:
                    ok = st.cond.wait_for(lambda: key in st.kv or st.closed, timeout=st.timeout)
                    val = st.kv.get(key) if ok else None
                if val is None:
                    self.wfile.write(b"\x01")
                    return
                self.wfile.write(b"\x00" + struct.pack(">I", len(val)) + val)
            else:
                return


class _StoreServer(socketserver.ThreadingTCPServer):
    daemon_threads = True
    allow_reuse_address = True


def _bind_address(host: str) -> str:
    """Where rank 0's store listens: MASTER_ADDR itself (loopback for bench.py's own
    launch), but every interface when the job spans nodes (WORLD_SIZE > LOCAL_WORLD_SIZE)
    and MASTER_ADDR resolves to a loopback address on this node (the common 127.0.1.1
    /etc/hosts entry), which peers on other nodes could not reach.
    WOST_STORE_BIND overrides it."""
    if os.environ.get("WOST_STORE_BIND") is not None:
        return os.environ["WOST_STORE_BIND"]
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    if world > local:
        try:
            if ipaddress.ip_address(socket.gethostbyname(host)).is_loopback:
                return ""
        except (OSError, ValueError):
            pass
    return host


class SocketStore:
    """A minimal key-value store over TCP (standard library only) for the communicator's
    id: rank 0 hosts it (``is_master``), every rank -- rank 0 too -- is a client. ``get``
    blocks until the key is set or ``timeout`` passes; keys are set once. The host listens
    on ``host`` itself (MASTER_ADDR: loopback for bench.py's own launch), not on every
    interface, and keeps serving until ``close`` (the communicator holds its store for
    its lifetime)."""

    def __init__(self, host: str, port: int, is_master: bool, timeout: float = 300.0):
        self.timeout = float(timeout)
        self._srv = self._f = self._sock = None
        if is_master:
            self.kv, self.cond, self.closed = {}, threading.Condition(), False
            self._srv = _StoreServer((_bind_address(host), int(port)), _StoreHandler)
            self._srv.store = self
            threading.Thread(target=self._srv.serve_forever, daemon=True).start()
        t0 = time.time()
        while True:   # the host may not listen yet
            try:
                self._sock = socket.create_connection((host, int(port)), timeout=self.timeout)
                break
            except OSError:
                if time.time() - t0 > self.timeout:
                    raise TimeoutError(f"no store at {host}:{port} after {self.timeout} s") from None
                time.sleep(0.05)
        self._sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        self._f = self._sock.makefile("rwb")

    @staticmethod
    def _lp(b: bytes) -> bytes:
        return struct.pack(">I", len(b)) + b

    def set(self, key: str, value: bytes):
        self._f.write(b"S" + self._lp(key.encode()) + self._lp(bytes(value)))
        self._f.flush()
        st = self._f.read(1)
        if st == b"\x01":
            raise KeyError(f"store: {key!r} is already set")
        if st != b"\x00":
            raise ConnectionError("store: set failed")

    def get(self, key: str) -> bytes:
        self._f.write(b"G" + self._lp(key.encode()))
        self._f.flush()
        st = self._f.read(1)
        if st != b"\x00":
            raise TimeoutError(f"store: no value for {key!r} within {self.timeout} s")
        n = struct.unpack(">I", self._f.read(4))[0]
        return self._f.read(n)

    def close(self):
        try:
            if getattr(self, "_f", None) is not None:
                self._f.close()
            if getattr(self, "_sock", None) is not None:
                self._sock.close()
        except OSError:
            pass
        self._f = self._sock = None
        if getattr(self, "_srv", None) is not None:
            with self.cond:
                self.closed = True
                self.cond.notify_all()
            self._srv.shutdown()
            self._srv.server_close()
            self._srv = None

    __del__ = close


class _FileStore:
    """Rank 0 publishes the id in a file named after values every rank of the launch
    shares (``tag``: MASTER_ADDR, MASTER_PORT -- the agent's store listens there, so the
    port is unique per live job on the node --, TORCHELASTIC_RUN_ID and the restart
    count), in a directory private to this user, and the others wait for it. The file is
    removed when rank 0's communicator closes (every rank has read it by then:
    ncclCommInitRank is collective). A file older than this process's start (less a
    minute of launch skew) is a crashed job's leftover and is not read."""

    def __init__(self, tag: str, rank: int, timeout: float):
        # a directory only this user can write, so no other user can plant an id there
        d = os.path.join(tempfile.gettempdir(), f"wost-{os.getuid()}")
        os.makedirs(d, mode=0o700, exist_ok=True)
        st = os.stat(d)
        if st.st_uid != os.getuid() or (st.st_mode & 0o022):
            raise PermissionError(f"{d} is not a private directory of this user")
        self.dir, self.tag, self.rank, self.timeout, self.paths = d, tag, rank, timeout, []
        start = _process_start_time()
        self.not_before = start - 60.0 if start is not None else 0.0   # (unknown start: the tag alone)

    def _path(self, key: str) -> str:
        safe = "".join(c if c.isalnum() else "_" for c in key)
        return os.path.join(self.dir, f"wost_uid.{self.tag}.{safe}")

    def set(self, key: str, value: bytes):
        path = self._path(key)
        tmp = f"{path}.tmp.{os.getpid()}"
        with open(tmp, "wb") as f:
            f.write(bytes(value))
        os.replace(tmp, path)
        self.paths.append(path)

    def get(self, key: str) -> bytes:
        path = self._path(key)
        t0 = time.time()
        while True:
            try:
                with open(path, "rb") as f:
                    if os.fstat(f.fileno()).st_mtime >= self.not_before:
                        return f.read()
            except OSError:
                pass
            if time.time() - t0 > self.timeout:
                raise TimeoutError(f"no communicator id in {path} after {self.timeout} s")
            time.sleep(0.02)

    def close(self):
        for p in self.paths:
            try:
                os.remove(p)
            except OSError:
                pass
        self.paths = []


def _process_start_time():
    """This process's start (wall clock, s): psutil, else /proc (the start in clock ticks
    after boot plus the boot time), else None -- then no staleness test beyond the tag
    (falling back to "now" made a late rank ignore a valid id file)."""
    try:
        import psutil

        return float(psutil.Process().create_time())
    except Exception:
        pass
    try:
        with open("/proc/self/stat") as f:
            ticks = float(f.read().rsplit(")", 1)[1].split()[19])   # field 22: starttime
        with open("/proc/stat") as f:
            btime = next(float(l.split()[1]) for l in f if l.startswith("btime"))
        return btime + ticks / os.sysconf("SC_CLK_TCK")
    except Exception:
        return None


def _launch_tag() -> str:
    """The file store's name for this launch: values every rank of it shares (not the
    parent pid -- a rank may sit below a wrapper of its own)."""
    parts = [os.environ.get("MASTER_ADDR", ""), os.environ.get("MASTER_PORT", "0"),
             os.environ.get("TORCHELASTIC_RUN_ID", ""), os.environ.get("TORCHELASTIC_RESTART_COUNT", "0")]
    return ".".join("".join(c if c.isalnum() else "_" for c in p) for p in parts)


def launch_store(timeout: float = 300.0):
    """The id exchange channel of this launch (module docstring): a SocketStore hosted by
    rank 0 on MASTER_PORT, a per-node file under torchrun's agent, or -- multi-node
    torchrun only -- torch's TCPStore client of the agent's store."""
    rank, world = int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1"))
    agent = os.environ.get("TORCHELASTIC_USE_AGENT_STORE", "").lower() == "true"
    if not agent:
        return SocketStore(os.environ.get("MASTER_ADDR", "127.0.0.1"), int(os.environ["MASTER_PORT"]),
                           is_master=(rank == 0), timeout=timeout)
    if int(os.environ.get("LOCAL_WORLD_SIZE", "0")) == world:   # one node: a file on it
        return _FileStore(_launch_tag(), rank, timeout)
    from datetime import timedelta

    import torch.distributed as dist

    return dist.TCPStore(os.environ.get("MASTER_ADDR", "127.0.0.1"), int(os.environ["MASTER_PORT"]), world,
                         is_master=False, timeout=timedelta(seconds=timeout))


def shard_walk_range(walks_per_point: int, n_ranks: int, rank: int) -> tuple[int, int]:
    """Rank `rank`'s walk range [begin, end) of each point (wost_shard_walk_range)."""
    nb = (int(walks_per_point) + _lib.WOST_BLOCK_WALKS - 1) // _lib.WOST_BLOCK_WALKS
    b0, b1 = nb * rank // n_ranks, nb * (rank + 1) // n_ranks
    return min(b0 * _lib.WOST_BLOCK_WALKS, walks_per_point), min(b1 * _lib.WOST_BLOCK_WALKS, walks_per_point)


def exchange_over_store(make_id, key: str = "wost_comm_uid", timeout: float = 300.0, store=None):
    """Rank 0 publishes make_id() under `key` in the launch's store (launch_store: no
    PyTorch unless a multi-node torchrun job), every rank reads it back: (bytes, store).
    The key is scoped by the run id and restart count, so a restarted job never reads a
    stale id. A further id (a second communicator) passes the first one's store."""
    rank = int(os.environ.get("RANK", "0"))
    if store is None:
        store = launch_store(timeout)
    k = f"{key}/{os.environ.get('TORCHELASTIC_RUN_ID', '')}/{os.environ.get('TORCHELASTIC_RESTART_COUNT', '0')}"
    if rank == 0:
        store.set(k, make_id())
    return bytes(store.get(k)), store


def unique_id() -> bytes:
    buf = (ctypes.c_uint8 * _lib.WOST_COMM_ID_BYTES)()
    _lib.check(_lib.lib.wost_comm_unique_id(buf), "wost_comm_unique_id", comm=True)
    return bytes(buf)


class Communicator:
    """An RCCL communicator of libwost (wost_comm_create)."""

    def __init__(self, uid: bytes, n_ranks: int, rank: int, device: int):
        if len(uid) != _lib.WOST_COMM_ID_BYTES:
            raise ValueError(f"unique id must be {_lib.WOST_COMM_ID_BYTES} bytes")
        buf = (ctypes.c_uint8 * _lib.WOST_COMM_ID_BYTES).from_buffer_copy(uid)
        h = ctypes.c_void_p()
        _lib.check(_lib.lib.wost_comm_create(buf, int(n_ranks), int(rank), int(device), ctypes.byref(h)),
                   "wost_comm_create", comm=True)
        self._c = h
        self.n_ranks, self.rank, self.device = int(n_ranks), int(rank), int(device)

    @classmethod
    def from_torch(cls, group=None, device: int | None = None) -> "Communicator":
        """Bootstrap over an initialised torch.distributed group (only the id travels)."""
        import torch.distributed as dist

        rank, world = dist.get_rank(group), dist.get_world_size(group)
        box = [unique_id() if rank == 0 else None]
        dist.broadcast_object_list(box, src=0, group=group)
        if device is None:
            device = int(os.environ.get("LOCAL_RANK", "0"))
        return cls(box[0], world, rank, device)

    @classmethod
    def from_env(cls, device: int | None = None, key: str = "wost_comm_uid", timeout: float = 300.0,
                 store=None) -> "Communicator":
        """Bootstrap from the torchrun environment (RANK, WORLD_SIZE, LOCAL_RANK, MASTER_ADDR,
        MASTER_PORT) without a torch process group: the id travels through a TCP
        key-value store (exchange_over_store). A further communicator over the same
        ranks passes its own ``key`` and the first one's ``_store``."""
        rank, world = int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1"))
        if device is None:
            device = int(os.environ.get("LOCAL_RANK", "0"))
        if world == 1 and "MASTER_PORT" not in os.environ:   # a lone process: no store needed
            return cls(unique_id(), 1, 0, device)
        own = store is None
        uid, store = exchange_over_store(unique_id, key, timeout, store)
        c = cls(uid, world, rank, device)
        c._store = store   # keep the store (and, on rank 0, its server) alive with the communicator
        c._owns_store = own
        return c

    @classmethod
    def from_file(cls, path: str, n_ranks: int, rank: int, device: int, timeout: float = 120.0) -> "Communicator":
        """Bootstrap through a file: rank 0 writes the id (atomically), the others wait for it.
        The caller removes a stale file before rank 0 starts."""
        if rank == 0:
            tmp = f"{path}.tmp.{os.getpid()}"
            with open(tmp, "wb") as f:
                f.write(unique_id())
            os.replace(tmp, path)
        t0 = time.time()
        while True:
            try:
                with open(path, "rb") as f:
                    uid = f.read()
                if len(uid) == _lib.WOST_COMM_ID_BYTES:
                    break
            except OSError:
                pass
            if time.time() - t0 > timeout:
                raise TimeoutError(f"no communicator id in {path} after {timeout} s")
            time.sleep(0.05)
        return cls(uid, n_ranks, rank, device)

    def close(self):
        if getattr(self, "_c", None) is not None and self._c.value:
            _lib.lib.wost_comm_destroy(self._c)
            self._c = None
        st = getattr(self, "_store", None)
        if st is not None and getattr(self, "_owns_store", False) and hasattr(st, "close"):
            st.close()
        self._store = None

    __del__ = close

    def allgather(self, a: np.ndarray) -> np.ndarray:
        """[n_ranks, *a.shape] float64: every rank's array, in rank order."""
        a = np.ascontiguousarray(a, np.float64)
        out = np.empty((self.n_ranks,) + a.shape, np.float64)
        _lib.check(_lib.lib.wost_comm_allgather(self._c, _lib.dptr(a), a.size, _lib.dptr(out)),
                   "wost_comm_allgather", comm=True)
        return out

    def allreduce(self, a, op: str = "sum") -> np.ndarray:
        ops = {"sum": _lib.WOST_COMM_SUM, "max": _lib.WOST_COMM_MAX}
        if op not in ops:
            raise ValueError(f"allreduce op must be 'sum' or 'max', got {op!r}")
        a = np.array(a, np.float64, copy=True, ndmin=1)
        _lib.check(_lib.lib.wost_comm_allreduce(self._c, _lib.dptr(a), a.size, ops[op]), "wost_comm_allreduce",
                   comm=True)
        return a

    def barrier(self):
        _lib.check(_lib.lib.wost_comm_barrier(self._c), "wost_comm_barrier", comm=True)


def _distributed_sums(solver, comm: Communicator, p: np.ndarray, nWalks: int, maxSteps: int, eps: float,
                      seed: int):
    n = p.shape[0]
    ns = ctypes.c_int32(1)
    _lib.check(_lib.lib.wost_num_sources(solver._h, ctypes.byref(ns)), "wost_num_sources")
    sums = np.zeros((n, 2 * ns.value + 1), np.float64)
    t = _lib.WostDistTiming()
    _lib.check(_lib.lib.wost_solve_distributed(solver._h, comm._c, _lib.fptr(p), n, int(nWalks), int(maxSteps),
                                               float(eps), int(seed) & (2**64 - 1), _lib.dptr(sums), ctypes.byref(t)),
               "wost_solve_distributed", comm=True)
    timing = {k: getattr(t.local, k) for k, _ in _lib.WostTiming._fields_}
    timing.update({"walk_begin": int(t.walk_begin), "walk_end": int(t.walk_end), "all_steps": int(t.total_steps),
                   "local_ms": float(t.local_ms), "agree_ms": float(t.agree_ms), "gather_ms": float(t.gather_ms),
                   "merge_ms": float(t.merge_ms)})
    solver.last_timing = timing
    solver.last_point_sums = sums
    return sums, timing


def solve_distributed(solver, comm: Communicator, points, nWalks: int, maxSteps: int = 1000, eps: float = 1e-4,
                      seed: int = 0):
    """WostSolver_2D.solve across the communicator's ranks (collective; every rank passes
    the same arguments). Returns (u [N,1] float32, SolveStats, timing dict) on every rank;
    u and the statistics are bitwise those of a one-GPU solve. Multi-source solves go
    through solve_sources_distributed."""
    from .solvers.WoStSolver import stats_from_sums

    p = np.ascontiguousarray(np.asarray(points, np.float32).reshape(-1, 2))
    sums, timing = _distributed_sums(solver, comm, p, nWalks, maxSteps, eps, seed)
    if sums.shape[1] != 3:
        raise ValueError("the solver scores several sources: use solve_sources_distributed")
    st = stats_from_sums(sums, int(nWalks), timing["all_steps"], timing["walk_kernel_ms"], timing["total_ms"])
    return st.mean.astype(np.float32).reshape(p.shape[0], 1), st, timing


def solve_sources_distributed(solver, comm: Communicator, points, sources, nWalks: int, maxSteps: int = 1000,
                              eps: float = 1e-4, seed: int = 0):
    """WostSolver_2D.solve_sources across the communicator's ranks (collective): every
    source scored by the same walks, the walk ranges sharded as in solve_distributed.
    Returns (u [S, N] float32, SolveStats with [S, N] mean / stderr, timing dict) on
    every rank, bitwise those of a one-GPU solve_sources."""
    from .solvers.WoStSolver import SolveStats, _stats_of_multi

    p = np.ascontiguousarray(np.asarray(points, np.float32).reshape(-1, 2))
    fields = solver.source_fields(sources)
    stats, steps, lsteps, kms, tms = [], 0, 0, 0.0, 0.0
    for c0 in range(0, len(fields), _lib.WOST_MAX_SOURCES):
        with solver.sources_installed(fields[c0:c0 + _lib.WOST_MAX_SOURCES]):
            sums, timing = _distributed_sums(solver, comm, p, nWalks, maxSteps, eps, seed)
        stats.extend(_stats_of_multi(sums, int(nWalks)))
        steps += timing["all_steps"]
        lsteps += timing["total_steps"]
        kms += timing["walk_kernel_ms"]
        tms += timing["total_ms"]
    timing = dict(timing, all_steps=steps, total_steps=lsteps, walk_kernel_ms=kms, total_ms=tms)
    solver.last_timing = timing
    u = np.stack([st.mean.astype(np.float32) for st in stats])
    return u, SolveStats(mean=np.stack([st.mean for st in stats]), stderr=np.stack([st.stderr for st in stats]),
                         mean_steps=stats[0].mean_steps, walks=int(nWalks), total_steps=steps, kernel_ms=kms,
                         total_ms=tms), timing
