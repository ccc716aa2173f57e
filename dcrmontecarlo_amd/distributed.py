"""Sharding arithmetic of multi-GPU solves, and a torch.distributed variant.

The product path is dcrmontecarlo_amd.comm: libwost's own RCCL communicator and
wost_solve_distributed (rank r solves the walk range shard_walk_range(W, R, r) of
every point, one all-gather of the block sums, per-point sums in global block
order -- bitwise the one-GPU result). This module holds the host-side mirror of
that merge (merge_walk_range_blocks, block_stats_of_walks: the gloo CPU tests
drive real shards of oracle walks through it), the weak-scaling replication
helpers of bench.py, and the torch.distributed path: libwost's own protocol
(wost_distributed_run -- the code wost_solve_distributed runs over RCCL) with
torch's collectives as its transport, for callers that already run a torch
process group, and for the gloo CPU tests of that protocol.
"""
from __future__ import annotations

import ctypes

import numpy as np

from .solvers.WoStSolver import stats_from_sums


def shard_walk_range(walks_per_point: int, world: int, rank: int) -> tuple[int, int]:
    """Rank `rank`'s walk range of every point: whole blocks, evenly split
    (wost_shard_walk_range; dcrmontecarlo_amd.comm.shard_walk_range)."""
    B = 4096   # WOST_BLOCK_WALKS
    nb = (int(walks_per_point) + B - 1) // B
    b0, b1 = nb * rank // world, nb * (rank + 1) // world
    return min(b0 * B, walks_per_point), min(b1 * B, walks_per_point)


def block_stats_of_walks(values: np.ndarray, steps: np.ndarray, walk_begin: int) -> np.ndarray:
    """(sum, sum^2, steps) of each WOST_BLOCK_WALKS block of per-walk values [N, Wr]
    whose first walk is walk_begin (block-aligned): [N, blocks, 3], summed in walk
    order (a host stand-in for the device reduction)."""
    B = 4096
    v = np.asarray(values, np.float64)
    s = np.asarray(steps, np.float64)
    n, wr = v.shape
    nb = (wr + B - 1) // B
    out = np.zeros((n, nb, 3))
    for b in range(nb):
        sl = slice(b * B, min((b + 1) * B, wr))
        out[:, b, 0] = v[:, sl].sum(1)
        out[:, b, 1] = (v[:, sl] ** 2).sum(1)
        out[:, b, 2] = s[:, sl].sum(1)
    return out


def merge_walk_range_blocks(parts, walks_per_point: int) -> np.ndarray:
    """Per-point sums from every rank's [N, blocks_r, 3] block rows (rank order): rank
    0's blocks, then rank 1's, ... -- the global block order of one GPU -- added to
    0.0 one block at a time, exactly as wost_solve_distributed does."""
    world = len(parts)
    n = parts[0].shape[0]
    acc = np.zeros((n, parts[0].shape[2]))
    for r in range(world):
        w0, w1 = shard_walk_range(walks_per_point, world, r)
        nb = (w1 - w0 + 4095) // 4096 if w1 > w0 else 0
        for b in range(nb):
            acc += parts[r][:, b]
    return acc


def shard_range(n_blocks: int, rank: int, world: int) -> tuple[int, int]:
    return rank * n_blocks // world, (rank + 1) * n_blocks // world


def gather_block_stats(local: np.ndarray, n_blocks: int, group=None, device=None) -> np.ndarray:
    """All ranks' [blocks, 3] float64 rows, concatenated in block order."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    n_max = (n_blocks + world - 1) // world + 1
    buf = torch.zeros((n_max, 3), dtype=torch.float64, device=device or "cpu")
    buf[: local.shape[0]] = torch.from_numpy(np.ascontiguousarray(local))
    outs = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(outs, buf, group=group)
    parts = []
    for r, o in enumerate(outs):
        b0, b1 = shard_range(n_blocks, r, world)
        parts.append(o[: b1 - b0].cpu().numpy())
    return np.concatenate(parts)


def point_sums(block_stats: np.ndarray, n_points: int) -> np.ndarray:
    """Per-point (sum, sum^2, steps) summed over blocks sequentially in block order --
    the same order as libwost's own point_stats, so single- and multi-GPU results
    agree bit for bit."""
    nbpp = block_stats.shape[0] // max(n_points, 1)
    b = block_stats.reshape(n_points, nbpp, 3)
    acc = np.zeros((n_points, 3), np.float64)
    for j in range(nbpp):
        acc += b[:, j]
    return acc


def replicate_points(points: np.ndarray, world: int) -> np.ndarray:
    """Weak scaling: the survey's points once per rank, [world * N, 2]. Copy r is
    points r*N .. r*N+N-1, so its walk ids (point * nWalks + walk) are distinct
    from every other copy's and, with the blocks sharded by shard_range, rank r
    solves exactly copy r: the one-GPU workload, on its own random streams."""
    p = np.ascontiguousarray(np.asarray(points, np.float32).reshape(-1, 2))
    return np.ascontiguousarray(np.tile(p, (world, 1)))


def merge_replicas(sums: np.ndarray, world: int) -> np.ndarray:
    """Per-point (sum, sum^2, steps) of replicate_points' copies merged in rank
    order: [world * N, 3] -> [N, 3], the statistics of world * nWalks walks per point."""
    n = sums.shape[0] // world
    b = sums.reshape(world, n, sums.shape[1])
    acc = np.zeros((n, sums.shape[1]), np.float64)
    for r in range(world):
        acc += b[r]
    return acc


class _Transport:
    """Python callables behind a wost_dist_ops (include/wost.h): libwost's own
    distributed protocol (wost_distributed_run) drives them. An exception in a
    callback becomes an error status for the protocol (and is re-raised by
    run_protocol on the rank where it happened)."""

    def __init__(self, n_points, row, solve_range, allreduce, allgather, prepare=None, n_ranks=None, key=None):
        from . import _lib

        self.error = None
        self.n_points, self.row = int(n_points), int(row)
        self.n_ranks = None if n_ranks is None else int(n_ranks)

        def guard(fn):
            def wrapped(*a):
                try:
                    return fn(*a)
                except Exception as e:   # noqa: BLE001 -- reported through the protocol
                    if self.error is None:
                        self.error = e
                    return _lib.WOST_ERR_COMM
            return wrapped

        def _solve(ctx, w0, w1, blocks):
            nbr = -(-(int(w1) - int(w0)) // _lib.WOST_BLOCK_WALKS)
            b = np.ascontiguousarray(solve_range(int(w0), int(w1)), np.float64)
            if b.shape != (self.n_points, nbr, self.row):
                raise ValueError(f"solve_range returned {b.shape}, expected {(self.n_points, nbr, self.row)}")
            ctypes.memmove(blocks, b.ctypes.data, b.nbytes)
            return 0

        def _allreduce(ctx, ptr, count, op):
            a = np.ctypeslib.as_array(ptr, shape=(int(count),))
            a[:] = allreduce(a.copy(), "sum" if op == _lib.WOST_COMM_SUM else "max")
            return 0

        def _allgather(ctx, send, count, recv):
            a = np.ctypeslib.as_array(send, shape=(int(count),)).copy()
            out = np.ascontiguousarray(allgather(a), np.float64).ravel()
            # recv holds n_ranks * count doubles: a transport whose group is not the
            # protocol's n_ranks must not write past it
            if self.n_ranks is not None and out.size != self.n_ranks * int(count):
                raise ValueError(f"allgather returned {out.size} values, expected {self.n_ranks} ranks x {int(count)}")
            r = np.ctypeslib.as_array(recv, shape=(out.size,))
            r[:] = out
            return 0

        def _prepare(ctx, count):
            if prepare is not None:
                prepare(int(count))
            return 0

        self._cb = (_lib.DIST_PREPARE(guard(_prepare)), _lib.DIST_SOLVE_RANGE(guard(_solve)),
                    _lib.DIST_ALLREDUCE(guard(_allreduce)), _lib.DIST_ALLGATHER(guard(_allgather)))
        self._key = None if key is None else np.ascontiguousarray(key, np.float64).ravel()
        self.ops = _lib.WostDistOps(None, *self._cb, _lib.dptr(self._key) if self._key is not None else None,
                                    0 if self._key is None else int(self._key.size))


def solve_key(seed: int, eps: float, max_steps: int, points) -> np.ndarray:
    """The agreement key of a solve (wost_dist_solve_key): seed halves, eps, maxSteps and
    a checksum of the float32 points -- values every rank must pass identically."""
    from . import _lib

    p = np.ascontiguousarray(np.asarray(points, np.float32).reshape(-1, 2))
    key = np.zeros(6, np.float64)
    _lib.check(_lib.lib.wost_dist_solve_key(int(seed) & (2**64 - 1), float(eps), int(max_steps), _lib.fptr(p),
                                            p.shape[0], _lib.dptr(key)), "wost_dist_solve_key")
    return key


def run_protocol(n_ranks: int, rank: int, n_points: int, walks_per_point: int, row: int, solve_range, allreduce,
                 allgather, prepare=None, key=None, phases: dict | None = None):
    """libwost's distributed protocol (wost_distributed_run: agreement all-reduce,
    all-gather of the padded block rows, ordered merge) over Python callables:
    solve_range(w0, w1) -> [n_points, blocks, row] float64 of this rank's walks;
    allreduce(a, "sum"|"max") -> a reduced; allgather(a) -> [n_ranks, a.size].
    ``key`` (optional, <= 16 values, e.g. solve_key(...)): arguments every rank must
    hold identically; a rank that differs makes every rank raise ValueError.
    Returns (point sums [n_points, row], (walk_begin, walk_end), total walk-steps).
    Raises the local exception on the rank whose callback failed, WostError on the
    others (no rank is left waiting in a collective). ``phases`` (a dict) receives the
    protocol's wall-clock phases on this rank (wost_dist_last_phases): local_ms (the
    local solve and pack), agree_ms (the agreement all-reduce: it waits for the slowest
    rank), gather_ms and merge_ms."""
    from . import _lib

    tr = _Transport(n_points, row, solve_range, allreduce, allgather, prepare, n_ranks=n_ranks, key=key)
    out = np.zeros((int(n_points), int(row)), np.float64)
    w0, w1, steps = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_uint64()
    rc = _lib.lib.wost_distributed_run(ctypes.byref(tr.ops), int(n_ranks), int(rank), int(n_points),
                                       int(walks_per_point), int(row), _lib.dptr(out), ctypes.byref(w0),
                                       ctypes.byref(w1), ctypes.byref(steps))
    if phases is not None:
        ms = (ctypes.c_double * 4)()
        _lib.lib.wost_dist_last_phases(ms)
        phases.update(local_ms=ms[0], agree_ms=ms[1], gather_ms=ms[2], merge_ms=ms[3])
    if rc != _lib.WOST_OK and tr.error is not None:
        raise tr.error
    _lib.check(rc, "wost_distributed_run", comm=True)
    return out, (int(w0.value), int(w1.value)), int(steps.value)


def torch_transport(group=None, device=None):
    """(allreduce, allgather) over a torch.distributed group (gloo on CPU; with
    ``device`` a CUDA device, the nccl/RCCL backend)."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    dev = device or "cpu"

    def allreduce(a, op):
        t = torch.from_numpy(np.ascontiguousarray(a, np.float64)).to(dev)
        dist.all_reduce(t, op=dist.ReduceOp.SUM if op == "sum" else dist.ReduceOp.MAX, group=group)
        return t.cpu().numpy()

    def allgather(a):
        t = torch.from_numpy(np.ascontiguousarray(a, np.float64)).to(dev)
        outs = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(outs, t, group=group)
        return np.stack([o.cpu().numpy() for o in outs])

    return allreduce, allgather


def solve_distributed(solver, points, nWalks: int, maxSteps: int = 1000, eps: float = 1e-4, seed: int = 0,
                      group=None, device=None):
    """WostSolver_2D.solve across the ranks of ``group`` (torch.distributed must be
    initialised): libwost's walk-range protocol (wost_distributed_run) with torch's
    collectives as the transport. Returns (u [N,1] float32, SolveStats) on every
    rank, bitwise those of a one-GPU solve."""
    import torch.distributed as dist

    pts = np.ascontiguousarray(np.asarray(points, np.float32).reshape(-1, 2))
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    ar, ag = torch_transport(group, device)
    sums, _, steps = run_protocol(world, rank, pts.shape[0], int(nWalks), 3,
                                  lambda w0, w1: solver.solve_range(pts, nWalks, w0, w1, maxSteps, eps, seed), ar, ag,
                                  key=solve_key(seed, eps, maxSteps, pts))
    u = (sums[:, 0] / nWalks).astype(np.float32).reshape(-1, 1)
    return u, stats_from_sums(sums, nWalks, steps)
