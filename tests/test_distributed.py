"""Multi-rank reduction with the gloo backend on CPU, world_size 2 and 3: shards
partition the blocks, the all_gather reassembles them in block order, and the
per-point sums are bitwise identical to one rank's. The merge and the failure
protocol are libwost's own C++ (wost_shard_pack / wost_shard_merge /
wost_distributed_run, the code wost_solve_distributed runs over RCCL), driven
here through gloo with oracle walk shards; no device is needed."""
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
class _NoTorch:
    """A meta-path finder that refuses every import of torch (the product bootstrap must
    not need it)."""

    def find_spec(self, name, path=None, target=None):
        if name == "torch" or name.startswith("torch."):
            raise ImportError(f"torch is blocked in this test ({name})")
        return None


def _store_worker(rank, world, port, mode, out_q):
    import sys

    if mode in ("socket", "agent_file"):
        for m in [m for m in sys.modules if m == "torch" or m.startswith("torch.")]:
            del sys.modules[m]
        sys.meta_path.insert(0, _NoTorch())
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from dcrmontecarlo_amd import comm

    agent = mode != "socket"
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                      TORCHELASTIC_RUN_ID="t1", TORCHELASTIC_USE_AGENT_STORE="True" if agent else "False",
                      LOCAL_WORLD_SIZE=str(world if mode == "agent_file" else 1))
    uid, store = comm.exchange_over_store(lambda: bytes(range(128)) if rank == 0 else b"wrong", timeout=60)
    out_q.put((rank, uid, "torch" in sys.modules, type(store).__name__))
    store.set(f"done{rank}", b"1")
    if rank == 0:   # the host of the store (or the writer of the file) outlives every reader
        for r in range(world):
            store.get(f"done{r}")
        if hasattr(store, "close"):
            store.close()


def _nested_store_worker(rank, world, port, out_q):
    """A rank below a wrapper process of its own (`--no-python` scripts, env
    wrappers): the ranks no longer share a parent."""
    ctx = mp.get_context("spawn")
    p = ctx.Process(target=_store_worker, args=(rank, world, port, "agent_file", out_q))
    p.start()
    p.join(timeout=120)
    raise SystemExit(p.exitcode)


@pytest.mark.parametrize("mode", ["socket", "agent_file", "agent_file_nested", "agent_tcp"])
def test_communicator_id_travels_through_the_launch_store(mode):
    """Communicator.from_env's id exchange (the part that needs no GPU): rank 0's 128 bytes
    reach every rank -- rank 0 hosting the standard-library socket store (bench.py's own
    launcher; torch import blocked), the ranks of one torchrun node meeting in a file
    (torch import blocked), or a multi-node torchrun agent's TCPStore."""
    from datetime import timedelta

    world = 3
    port = _free_port()
    host = dist.TCPStore("127.0.0.1", port, None, is_master=True, timeout=timedelta(seconds=60),
                         wait_for_workers=False) if mode == "agent_tcp" else None
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    if mode == "agent_file_nested":
        procs = [ctx.Process(target=_nested_store_worker, args=(r, world, port, q)) for r in range(world)]
    else:
        procs = [ctx.Process(target=_store_worker, args=(r, world, port, mode, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {r: rest for r, *rest in (q.get(timeout=120) for _ in range(world))}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(res[r][0] == bytes(range(128)) for r in range(world))
    want = {"socket": "SocketStore", "agent_file": "_FileStore", "agent_file_nested": "_FileStore",
            "agent_tcp": "TCPStore"}[mode]
    assert all(res[r][2] == want for r in range(world)), res
    if mode != "agent_tcp":
        assert not any(res[r][1] for r in range(world)), "torch was imported"
    del host


# ---------------------------------------------------------------- libwost's C++ merge and protocol
def _lib_pack_merge(parts_blocks, W, R, row):
    """Pack every rank's blocks with wost_shard_pack, concatenate (the all-gather's
    layout) and merge with wost_shard_merge."""
    from dcrmontecarlo_amd import _lib

    n = parts_blocks[0].shape[0]
    nb_max = int(_lib.lib.wost_shard_blocks_max(W, R))
    gathered = np.zeros((R, n, nb_max, row))
    for r in range(R):
        b = np.ascontiguousarray(parts_blocks[r], np.float64)
        out = np.empty((n, nb_max, row))
        assert _lib.lib.wost_shard_pack(_lib.dptr(b), n, W, R, r, row, _lib.dptr(out)) == 0
        gathered[r] = out
    sums = np.empty((n, row))
    assert _lib.lib.wost_shard_merge(_lib.dptr(gathered), n, W, R, row, _lib.dptr(sums)) == 0
    return sums


@pytest.mark.parametrize("row", [3, 7])
@pytest.mark.parametrize("W", [1, 4096, 3 * 4096 + 1000, 11 * 4096, 20 * 4096 + 1])
def test_library_merge_equals_mirror_and_one_rank(W, row):
    """wost_shard_pack + wost_shard_merge (the C++ of wost_solve_distributed) for
    R in {2, 3, 8}, ragged last shards, empty shards (R > blocks) and multi-source
    rows (2S+1 = 7): bitwise equal to the host mirror and to one rank's sums."""
    rng = np.random.default_rng(W + row)
    n = 5
    nb = -(-W // 4096)
    full = rng.standard_normal((n, nb, row)) * np.array([1e3, 1e-7, 1e6, 3.0, 1.0, 7.0, 4096.0][:row])
    one = _lib_pack_merge([full], W, 1, row)
    acc = np.zeros((n, row))
    for b in range(nb):      # one GPU: blocks of a point added to 0.0 in order
        acc += full[:, b]
    assert np.array_equal(one, acc)
    for R in (2, 3, 8):
        parts = []
        for r in range(R):
            w0, w1 = D.shard_walk_range(W, R, r)
            b0, b1 = w0 // 4096, -(-w1 // 4096) if w1 > w0 else w0 // 4096
            parts.append(full[:, b0:b1])
        got = _lib_pack_merge(parts, W, R, row)
        assert np.array_equal(got, acc), R
        assert np.array_equal(got, D.merge_walk_range_blocks(
            [np.pad(p, ((0, 0), (0, max(0, -(-nb // R) - p.shape[1])), (0, 0))) for p in parts], W))


def _protocol_worker(rank, world, port, W, mode, out_q):
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from dcrmontecarlo_amd import scenarios as S
    from dcrmontecarlo_amd import _lib

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sc = S.poisson_square()
    pts = sc.points[:3]
    ar, ag = D.torch_transport()

    myW = W + 4096 if (mode == "disagree" and rank == 1) else W
    seed = 100 if (mode == "disagree_seed" and rank == 1) else 99
    key = D.solve_key(seed, sc.eps, sc.max_steps, pts) if mode.startswith("disagree_") or mode == "ok" else None
    if mode == "nan_eps":   # every rank passes the same NaN: still no agreement
        key = D.solve_key(seed, float("nan"), sc.max_steps, pts)

    def solve_range(w0, w1):
        if mode == "fail" and rank == world - 1:
            raise RuntimeError("injected failure")
        return _oracle_range_blocks(sc, pts, myW, w0, w1, 99)

    try:
        sums, rng_, steps = D.run_protocol(world, rank, len(pts), myW, 3, solve_range, ar, ag, key=key)
        res = ("ok", sums, rng_, steps)
    except RuntimeError as e:
        res = (type(e).__name__, str(e), None, None)
    except ValueError as e:
        res = ("ValueError", str(e), None, None)
    out_q.put((rank, res))
    dist.barrier()          # every rank got here: nobody hangs in a collective
    dist.destroy_process_group()


def _run_protocol_world(world, W, mode):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_protocol_worker, args=(r, world, port, W, mode, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


@pytest.mark.parametrize("world", [2, 3])
def test_library_protocol_over_gloo_with_oracle_shards(world):
    """wost_distributed_run over gloo: rank r's walk range of every point comes from
    the CPU oracle (the device's Philox streams), the C++ agreement all-reduce,
    padded all-gather and ordered merge give one rank's sums bit for bit on every
    rank, and total_steps counts every rank's walk-steps."""
    from dcrmontecarlo_amd import scenarios as S

    W = 3 * 4096 + 1000
    res = _run_protocol_world(world, W, "ok")
    sc = S.poisson_square()
    single = D.merge_walk_range_blocks([_oracle_range_blocks(sc, sc.points[:3], W, 0, W, 99)], W)
    for r in range(world):
        status, sums, (w0, w1), steps = res[r]
        assert status == "ok"
        assert np.array_equal(sums, single)
        assert (w0, w1) == D.shard_walk_range(W, world, r)
        assert steps == int(single[:, 2].sum())


def test_library_protocol_failure_on_one_rank_reaches_every_rank():
    """a rank whose local solve fails still takes part in the agreement
    collective, so every rank returns an error instead of waiting in the gather:
    the failing rank re-raises its own exception, the others get WostError."""
    res = _run_protocol_world(2, 2 * 4096, "fail")
    assert res[1][0] == "RuntimeError" and "injected failure" in res[1][1]
    assert res[0][0] == "WostError" and "another rank failed" in res[0][1]


@pytest.mark.parametrize("mode", ["disagree", "disagree_seed"])
def test_library_protocol_rejects_disagreeing_ranks(mode):
    """Ranks called with different walk counts, or with different arguments in the
    agreement key (here the seed: wost_dist_solve_key), agree to fail (ValueError on all)."""
    res = _run_protocol_world(2, 2 * 4096, mode)
    for r in range(2):
        assert res[r][0] == "ValueError" and "disagree" in res[r][1], res[r]
    if mode == "disagree_seed":
        assert "arguments" in res[0][1]


def test_library_protocol_refuses_a_nan_argument_on_every_rank():
    """A NaN in the agreement key (here eps, the same NaN on every rank) cannot be agreed
    on: each rank fails it locally and every rank returns ValueError."""
    res = _run_protocol_world(2, 2 * 4096, "nan_eps")
    for r in range(2):
        assert res[r][0] == "ValueError" and "NaN" in res[r][1], res[r]


def test_solve_key_covers_seed_eps_steps_and_points():
    from dcrmontecarlo_amd import scenarios as S

    pts = S.poisson_square().points[:5]
    k = D.solve_key(2**40 + 7, 1e-4, 500, pts)
    assert k[0] == 7 and k[1] == 2**8 and k[2] == np.float32(1e-4) and k[3] == 500
    p2 = pts.copy()
    p2[3, 1] = np.nextafter(p2[3, 1], np.float32(9))
    assert not np.array_equal(k[4:], D.solve_key(2**40 + 7, 1e-4, 500, p2)[4:])
    assert np.array_equal(k, D.solve_key(2**40 + 7, 1e-4, 500, pts.astype(np.float64)))


def test_library_protocol_eight_thread_ranks_with_oracle_shards():
    """R = 8 (the driver's node size) through wost_distributed_run with thread ranks:
    oracle walk shards of 3 points, ragged (W not a multiple of 8 blocks, some ranks
    empty), one rank's sums on every rank."""
    from dcrmontecarlo_amd import scenarios as S
    from rank_threads import RankThreads

    sc = S.poisson_square()
    pts = sc.points[:3]
    W = 5 * 4096 + 17                       # 6 blocks over 8 ranks: two ranks hold none
    full = _oracle_range_blocks(sc, pts, W, 0, W, 5)
    single = D.merge_walk_range_blocks([full], W)
    R = 8

    def shard(w0, w1):
        return full[:, w0 // 4096:-(-w1 // 4096)]

    res = RankThreads(R).run(lambda r, ar, ag: D.run_protocol(R, r, len(pts), W, 3, shard, ar, ag))
    assert sum(1 for r in range(R) if res[r][1][0] == res[r][1][1]) == 2
    for r in range(R):
        assert np.array_equal(res[r][0], single)


def test_socket_store_is_set_once_bounded_and_local():
    """the store listens on MASTER_ADDR only, refuses a second set of a key
    (no peer can replace rank 0's id) and drops a request whose length prefix exceeds its
    cap instead of allocating it."""
    import socket
    import struct

    from dcrmontecarlo_amd import comm

    port = _free_port()
    st = comm.SocketStore("127.0.0.1", port, is_master=True, timeout=10)
    try:
        assert st._srv.server_address[0] == "127.0.0.1"
        st.set("id", b"abc")
        with pytest.raises(KeyError):
            st.set("id", b"evil")
        assert st.get("id") == b"abc"
        with socket.create_connection(("127.0.0.1", port), timeout=10) as c:
            c.sendall(b"S" + struct.pack(">I", 3) + b"big" + struct.pack(">I", 1 << 31))
            assert c.recv(1) == b""          # the server closed the connection
        assert st.get("id") == b"abc"
    finally:
        st.close()
