"""Sharding arithmetic of multi-GPU solves, and a torch.distributed variant.

The product path is dcrmontecarlo_amd.comm: libwost's own RCCL communicator and
wost_solve_distributed (rank r solves the walk range shard_walk_range(W, R, r) of
every point, one all-gather of the block sums, per-point sums in global block
order -- bitwise the one-GPU result). This module holds the host-side mirror of
that merge (merge_walk_range_blocks, block_stats_of_walks: the gloo CPU tests
drive real shards of oracle walks through it), the weak-scaling replication
helpers of bench.py, and an optional torch.distributed path (contiguous block
ranges, all_gather of the rows through torch's backend) for callers that
already run a torch process group.
"""
from __future__ import annotations

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


def solve_distributed(solver, points, nWalks: int, maxSteps: int = 1000, eps: float = 1e-4, seed: int = 0,
                      group=None, device=None):
    """WostSolver_2D.solve across the ranks of ``group`` (torch.distributed must be
    initialised). Returns (u [N,1] float32, SolveStats) on every rank."""
    import torch.distributed as dist

    pts = np.ascontiguousarray(np.asarray(points, np.float32).reshape(-1, 2))
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    nb = solver.num_blocks(pts.shape[0], nWalks)
    b0, b1 = shard_range(nb, rank, world)
    local = solver.solve_blocks(pts, nWalks, b0, b1, maxSteps, eps, seed)
    allb = gather_block_stats(local, nb, group, device)
    sums = point_sums(allb, pts.shape[0])
    u = (sums[:, 0] / nWalks).astype(np.float32).reshape(-1, 1)
    return u, stats_from_sums(sums, nWalks)
