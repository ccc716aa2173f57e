"""Multi-rank reduction (dcrmontecarlo_amd.distributed) with the gloo backend on CPU,
world_size 2 and 3: shards partition the blocks, the all_gather reassembles them
in block order, and the per-point sums are bitwise identical to one rank's."""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

from dcrmontecarlo_amd import distributed as D  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _block_rows(b0, b1):
    # deterministic synthetic block partials with awkward magnitudes
    j = np.arange(b0, b1, dtype=np.float64)
    return np.stack([np.sin(j) * 1e3 + 1e-7 * j, np.cos(j) ** 2 * 1e6, 4096.0 * (j % 7)], axis=1)


def _worker(rank, world, port, n_points, nbpp, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    nb = n_points * nbpp
    b0, b1 = D.shard_range(nb, rank, world)
    allb = D.gather_block_stats(_block_rows(b0, b1), nb)
    out_q.put((rank, D.point_sums(allb, n_points)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_gather_matches_single_rank(world):
    n_points, nbpp = 5, 7
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_points, nbpp, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    single = D.point_sums(_block_rows(0, n_points * nbpp), n_points)
    for r in range(world):
        assert np.array_equal(res[r], single)


def test_replicas_shard_one_copy_per_rank_and_merge():
    pts = np.arange(10, dtype=np.float32).reshape(5, 2)
    for world in (1, 2, 3, 8):
        rep = D.replicate_points(pts, world)
        assert rep.shape == (5 * world, 2) and np.array_equal(rep[5 * (world - 1):], pts)
        for nbpp in (1, 3, 245):
            nb = rep.shape[0] * nbpp
            for r in range(world):   # rank r's blocks are exactly copy r's
                assert D.shard_range(nb, r, world) == (r * 5 * nbpp, (r + 1) * 5 * nbpp)
        rows = np.stack([np.arange(5 * world, dtype=np.float64)] * 3, axis=1)
        m = D.merge_replicas(rows, world)
        assert np.array_equal(m[:, 0], sum(np.arange(5) + 5 * r for r in range(world)))


def test_shard_ranges_partition_blocks():
    for nb in (1, 7, 48 * 245):
        for world in (1, 2, 3, 8):
            ranges = [D.shard_range(nb, r, world) for r in range(world)]
            assert ranges[0][0] == 0 and ranges[-1][1] == nb
            assert all(a[1] == b[0] for a, b in zip(ranges, ranges[1:]))


# ---------------------------------------------------------------- walk-range shards of real walks
# the layout of libwost's wost_solve_distributed (dcrmontecarlo_amd.comm): rank r solves
# walks shard_walk_range(W, R, r) of EVERY point; here the walks are the CPU oracle's
# (same Philox streams as the device), the rows travel through gloo, and the merge is the
# host mirror of the library's
def _oracle_range_blocks(sc, pts, W, w0, w1, seed):
    from oracle import oracle as O

    pb = O.Problem.from_scenario(sc)
    vals, steps = [], []
    for p in range(len(pts)):
        v, s = pb.solve_walks(pts, W, sc.max_steps, sc.eps, seed, wid_begin=p * W + w0, wid_end=p * W + w1,
                              threads=1)
        vals.append(v)
        steps.append(s)
    return D.block_stats_of_walks(np.array(vals), np.array(steps), w0)


def _range_worker(rank, world, port, W, out_q):
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from dcrmontecarlo_amd import scenarios as S

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sc = S.poisson_square()
    pts = sc.points[:3]
    w0, w1 = D.shard_walk_range(W, world, rank)
    mine = _oracle_range_blocks(sc, pts, W, w0, w1, 99)
    nb_max = -(-(-(-W // 4096)) // world)
    pad = np.zeros((len(pts), nb_max, 3))
    pad[:, :mine.shape[1]] = mine
    outs = [torch.empty(pad.shape, dtype=torch.float64) for _ in range(world)]
    dist.all_gather(outs, torch.from_numpy(pad))
    parts = [o.numpy() for o in outs]
    out_q.put((rank, D.merge_walk_range_blocks(parts, W)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_walk_range_shards_of_oracle_walks_merge_to_one_rank(world):
    """Every rank solves its walk range of every point (oracle walks), the padded block
    rows are all-gathered, and the merged per-point sums equal one rank's bit for bit;
    the shards cover every walk exactly once."""
    from dcrmontecarlo_amd import scenarios as S

    W = 3 * 4096 + 1000
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_range_worker, args=(r, world, port, W, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    sc = S.poisson_square()
    single = D.merge_walk_range_blocks([_oracle_range_blocks(sc, sc.points[:3], W, 0, W, 99)], W)
    for r in range(world):
        assert np.array_equal(res[r], single)
    ranges = [D.shard_walk_range(W, world, r) for r in range(world)]
    assert ranges[0][0] == 0 and ranges[-1][1] == W and all(a[1] == b[0] for a, b in zip(ranges, ranges[1:]))
    assert all(a % 4096 == 0 for a, _ in ranges)
    assert np.all(single[:, 2] >= W)                  # every walk took at least one step


def test_walk_range_shards_match_the_library():
    """The host mirror of the shard arithmetic equals libwost's (no device needed)."""
    import ctypes

    from dcrmontecarlo_amd import _lib
    from dcrmontecarlo_amd import comm

    for W in (1, 4095, 4096, 12288, 1_000_000, 1 << 20):
        for R in (1, 2, 3, 4, 8):
            for r in range(R):
                a, b = ctypes.c_int64(), ctypes.c_int64()
                assert _lib.lib.wost_shard_walk_range(W, R, r, ctypes.byref(a), ctypes.byref(b)) == 0
                assert (a.value, b.value) == D.shard_walk_range(W, R, r) == comm.shard_walk_range(W, R, r)


# ---------------------------------------------------------------- communicator bootstrap
def _store_worker(rank, world, port, agent, out_q):
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from dcrmontecarlo_amd import comm

    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                      TORCHELASTIC_RUN_ID="t1", TORCHELASTIC_USE_AGENT_STORE="True" if agent else "False")
    uid, store = comm.exchange_over_store(lambda: bytes(range(128)) if rank == 0 else b"wrong", timeout=60)
    out_q.put((rank, uid))
    store.set(f"done{rank}", b"1")
    if rank == 0 and not agent:   # the host of the store outlives every reader
        for r in range(world):
            store.get(f"done{r}")


@pytest.mark.parametrize("agent", [False, True])
def test_communicator_id_travels_through_the_launch_store(agent):
    """Communicator.from_env's id exchange (the part that needs no GPU): rank 0's 128 bytes
    reach every rank, with rank 0 hosting the store or torchrun's agent hosting it."""
    from datetime import timedelta

    world = 3
    port = _free_port()
    host = dist.TCPStore("127.0.0.1", port, None, is_master=True, timeout=timedelta(seconds=60),
                         wait_for_workers=False) if agent else None
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_store_worker, args=(r, world, port, agent, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(res[r] == bytes(range(128)) for r in range(world))
    del host
