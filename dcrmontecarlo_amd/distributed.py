"""Multi-GPU solve: one process per GPU, walk blocks sharded, one RCCL collective.

The walks of a solve are grouped in blocks of WOST_BLOCK_WALKS consecutive
walks of one point (global walk id = point * nWalks + walk). Rank r of R
solves the contiguous block range [r*NB/R, (r+1)*NB/R) on its own GPU; the
per-block (sum, sum of squares, steps) rows are exchanged with one
``all_gather`` (backend "nccl" = RCCL over xGMI on MI355X, "gloo" on CPU for
tests) and every rank sums them per point in block order. Random streams are
keyed by global walk id, so the result is bitwise identical for any R.
"""
from __future__ import annotations

import numpy as np

from .solvers.WoStSolver import stats_from_sums


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
