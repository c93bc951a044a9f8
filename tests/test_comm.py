"""Reassembly transport (mando_comm_*): host-socket backend with several CPU ranks.

The RCCL backend is the same entry points bound to a device context (tests/test_define_gpu.py runs the
single-rank path on the GPU; multi-GPU runs come from the driver's scaling bench)."""
import multiprocessing as mp
import socket

import numpy as np
import pytest


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, q):
    from mandalorion_amd.comm import Comm

    with Comm(world, rank, "127.0.0.1", port, timeout_s=60) as c:
        blob = np.full(rank * 1000 + 3, rank + 1, dtype=np.uint8) if rank != 1 else np.zeros(0, np.uint8)
        allb, counts = c.allgather_bytes(blob)
        g, gc = c.gather_bytes(blob)
        assert gc.tolist() == counts.tolist()
        assert (g is None) == (rank != 0) and (g is None or g.tobytes() == allb.tobytes())
        m = c.max(float(rank) * 1.5)
        c.barrier()
        q.put((rank, counts.tolist(), allb.tobytes(), m, c.backend))


@pytest.mark.parametrize("world", [2, 3])
def test_host_allgather(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_rank, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = sorted(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    sizes = [0 if r == 1 else r * 1000 + 3 for r in range(world)]
    want = b"".join(bytes([r + 1]) * sizes[r] for r in range(world))
    for rank, counts, allb, m, backend in out:
        assert counts == sizes
        assert allb == want
        assert m == 1.5 * (world - 1)
        assert backend == "host"


def test_single_rank_needs_no_peers():
    from mandalorion_amd.comm import Comm

    with Comm(1, 0) as c:
        b, cnt = c.allgather_bytes(np.arange(10, dtype=np.uint8))
        assert cnt.tolist() == [10] and b.tolist() == list(range(10))
        g, gc = c.gather_bytes(np.arange(7, dtype=np.uint8))
        assert gc.tolist() == [7] and g.tolist() == list(range(7))
        assert c.max(2.5) == 2.5
        c.barrier()


def test_bad_arguments():
    from mandalorion_amd import _lib
    from mandalorion_amd.comm import Comm

    with pytest.raises(_lib.MandoError):
        Comm(2, 5, "127.0.0.1", 1234)


def _ragged_blob(rank: int) -> np.ndarray:
    """The multi-rank tests' payloads: ragged sizes, rank 1 sends nothing."""
    if rank == 1:
        return np.zeros(0, np.uint8)
    return ((np.arange(rank * 70001 + 13) * (rank + 3)) % 251).astype(np.uint8)


def _host_ragged_rank(rank, world, port, q):
    from mandalorion_amd.comm import Comm

    with Comm(world, rank, "127.0.0.1", port, timeout_s=60) as c:
        allb, counts = c.allgather_bytes(_ragged_blob(rank))
        g, _ = c.gather_bytes(_ragged_blob(rank))
        q.put((rank, counts.tolist(), allb.tobytes(), None if g is None else g.tobytes()))


def _rccl_replay(world: int, counts: list) -> tuple:
    """Replays the RCCL paths of mando_allgather_bytes / mando_gather_bytes (comm.hip) on host buffers from
    the library's own marshalling (mando_rccl_*_plan): ncclAllGather of maxc-padded slices, the per-rank
    compaction, and rank 0's point-to-point receives plus its device-to-host copy.  Padding and untouched
    device bytes are 0xEE, so a wrong offset or length shows up as foreign bytes."""
    import ctypes

    from mandalorion_amd import _lib

    lib = _lib.load()
    P = ctypes.c_void_p
    cnt = np.asarray(counts, np.int64)
    blobs = [_ragged_blob(r) for r in range(world)]
    assert [b.size for b in blobs] == counts
    # all-gather (every rank runs the same plan)
    maxc = np.zeros(1, np.int64)
    dev_off, host_off = np.zeros(world, np.int64), np.zeros(world, np.int64)
    assert lib.mando_rccl_allgather_plan(world, P(cnt.ctypes.data), P(maxc.ctypes.data), P(dev_off.ctypes.data),
                                         P(host_off.ctypes.data)) == 0
    m = int(maxc[0])
    assert m >= max(counts) and m >= 1
    drecv = np.full(m * world, 0xEE, np.uint8)
    for r in range(world):  # ncclAllGather: rank r's maxc-byte send buffer lands at r * maxc
        dsend = np.full(m, 0xEE, np.uint8)
        dsend[:counts[r]] = blobs[r]
        drecv[r * m:(r + 1) * m] = dsend
    allb = np.full(int(cnt.sum()), 0xEE, np.uint8)
    for r in range(world):
        allb[host_off[r]:host_off[r] + counts[r]] = drecv[dev_off[r]:dev_off[r] + counts[r]]
    # gather to rank 0: every rank's plan; sends and receives must pair up
    plans = []
    for rank in range(world):
        po, pl, d2 = np.zeros(world, np.int64), np.zeros(world, np.int64), np.zeros(2, np.int64)
        assert lib.mando_rccl_gather_plan(world, rank, P(cnt.ctypes.data), P(po.ctypes.data), P(pl.ctypes.data),
                                          P(d2.ctypes.data), P(d2.ctypes.data + 8)) == 0
        plans.append((po, pl, d2))
    tot = int(cnt.sum())
    d0 = np.full(max(tot, 1), 0xEE, np.uint8)
    for p in range(1, world):
        _, pl_p, d2_p = plans[p]
        assert pl_p[0] == counts[p] and not pl_p[1:].any() and not d2_p.any()  # a peer only sends, to 0
        assert plans[0][1][p] == pl_p[0]  # rank 0 posts the matching receive
        if pl_p[0]:
            d0[plans[0][0][p]:plans[0][0][p] + pl_p[0]] = blobs[p]
    assert plans[0][1][0] == 0  # rank 0 does not receive from itself
    g = np.full(tot, 0xEE, np.uint8)
    g[:counts[0]] = blobs[0]  # rank 0's own bytes stay on the host
    o, n = plans[0][2]
    g[o:o + n] = d0[o:o + n]
    return allb.tobytes(), g.tobytes()


@pytest.mark.parametrize("world", [2, 3])
def test_rccl_marshalling_equals_host_transport(world):
    """CPU-side check of the RCCL argument marshalling (counts, offsets, recv_counts): the RCCL paths'
    plans, replayed on host buffers, give the same bytes as the host transport run with `world` ranks."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_host_ragged_rank, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = sorted(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    counts = out[0][1]
    allb, g = _rccl_replay(world, counts)
    for rank, c, host_all, host_g in out:
        assert c == counts
        assert host_all == allb
        assert (host_g is None) == (rank != 0)
    assert out[0][3] == g


def test_rccl_plan_edge_cases():
    """Every rank empty (the padded all-gather still moves one byte per rank) and bad arguments."""
    import ctypes

    from mandalorion_amd import _lib

    lib = _lib.load()
    P = ctypes.c_void_p
    cnt = np.zeros(3, np.int64)
    maxc, a, b = np.zeros(1, np.int64), np.zeros(3, np.int64), np.zeros(3, np.int64)
    assert lib.mando_rccl_allgather_plan(3, P(cnt.ctypes.data), P(maxc.ctypes.data), P(a.ctypes.data),
                                         P(b.ctypes.data)) == 0
    assert maxc[0] == 1 and a.tolist() == [0, 1, 2] and b.tolist() == [0, 0, 0]
    d2 = np.zeros(2, np.int64)
    assert lib.mando_rccl_gather_plan(3, 0, P(cnt.ctypes.data), P(a.ctypes.data), P(b.ctypes.data),
                                      P(d2.ctypes.data), P(d2.ctypes.data + 8)) == 0
    assert b.tolist() == [0, 0, 0] and d2.tolist() == [0, 0]
    assert lib.mando_rccl_gather_plan(3, 3, P(cnt.ctypes.data), P(a.ctypes.data), P(b.ctypes.data),
                                      P(d2.ctypes.data), P(d2.ctypes.data + 8)) != 0
    cnt[1] = -1
    assert lib.mando_rccl_allgather_plan(3, P(cnt.ctypes.data), P(maxc.ctypes.data), P(a.ctypes.data),
                                         P(b.ctypes.data)) != 0


def _a2a_part(src: int, dst: int) -> np.ndarray:
    """The alltoallv tests' part from rank src to rank dst (ragged; rank 1 sends nothing to rank 0)."""
    if (src, dst) == (1, 0):
        return np.zeros(0, np.uint8)
    return ((np.arange(src * 3001 + dst * 17 + 5) * (src + 2 * dst + 1)) % 251).astype(np.uint8)


def _host_a2a_rank(rank, world, port, q):
    from mandalorion_amd.comm import Comm

    with Comm(world, rank, "127.0.0.1", port, timeout_s=60) as c:
        got = c.alltoallv([_a2a_part(rank, d) for d in range(world)])
        q.put((rank, [g.tobytes() for g in got]))


@pytest.mark.parametrize("world", [2, 3])
def test_host_alltoallv_and_rccl_plan(world):
    """alltoallv over the host transport (one all-gather, each rank keeps its parts), and the RCCL path's
    marshalling (mando_rccl_alltoallv_plan: offsets of each rank's part in the send and receive buffers)
    replayed on host buffers: the same bytes."""
    import ctypes

    from mandalorion_amd import _lib

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_host_a2a_rank, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = dict(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    lib = _lib.load()
    P = ctypes.c_void_p
    # the RCCL path: every rank's send buffer and offsets from the plan; rank d receives from rank s the
    # bytes at send_off[s][d] of s's buffer, into recv_off[d][s] of its own
    sends, soffs, roffs, rcs = [], [], [], []
    for r in range(world):
        parts = [_a2a_part(r, d) for d in range(world)]
        sc = np.array([p.size for p in parts], np.int64)
        rc = np.array([_a2a_part(s, r).size for s in range(world)], np.int64)
        so, ro = np.zeros(world, np.int64), np.zeros(world, np.int64)
        assert lib.mando_rccl_alltoallv_plan(world, P(sc.ctypes.data), P(rc.ctypes.data), P(so.ctypes.data),
                                             P(ro.ctypes.data)) == 0
        sends.append(np.concatenate(parts))
        soffs.append(so)
        roffs.append(ro)
        rcs.append(rc)
    for d in range(world):
        recv = np.full(int(rcs[d].sum()), 0xEE, np.uint8)
        for s_ in range(world):
            n = int(rcs[d][s_])
            recv[roffs[d][s_]:roffs[d][s_] + n] = sends[s_][soffs[s_][d]:soffs[s_][d] + n]
        replay = [recv[roffs[d][s_]:roffs[d][s_] + rcs[d][s_]].tobytes() for s_ in range(world)]
        want = [_a2a_part(s_, d).tobytes() for s_ in range(world)]
        assert out[d] == want
        assert replay == want


@pytest.mark.gpu
def test_rccl_backend_single_rank(gpu_ctx):
    """The RCCL path of mando_comm_init on the box's one GPU (ncclUniqueId drawn by rank 0,
    ncclCommInitRank on the ctx's device); multi-rank RCCL runs come from the driver's 8-GPU bench."""
    from mandalorion_amd.comm import Comm

    with Comm(1, 0, device_ctx=gpu_ctx) as c:
        assert c.backend == "rccl"
        b, cnt = c.allgather_bytes((np.arange(1000) % 251).astype(np.uint8))
        assert cnt.tolist() == [1000] and b.tolist() == [i % 251 for i in range(1000)]
        g, gc = c.gather_bytes((np.arange(999) % 13).astype(np.uint8))
        assert gc.tolist() == [999] and g.tolist() == [i % 13 for i in range(999)]
        a = c.alltoallv([(np.arange(777) % 7).astype(np.uint8)])
        assert len(a) == 1 and a[0].tolist() == [i % 7 for i in range(777)]
        c.barrier()


def _rccl_rank(rank, world, port, q):
    import os

    os.environ.update(WORLD_SIZE=str(world), RANK=str(rank), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    from mandalorion_amd.comm import Comm

    c = Comm.from_env(device=rank)
    try:
        # ragged sizes (rank 1 sends nothing): the padded ncclAllGather + per-slice compaction
        blob = _ragged_blob(rank)
        allb, counts = c.allgather_bytes(blob)
        # the writer's gather: point-to-point sends to rank 0 (ragged, one empty)
        g, gc = c.gather_bytes(blob)
        assert gc.tolist() == counts.tolist()
        assert (g is None) == (rank != 0) and (g is None or g.tobytes() == allb.tobytes())
        m = c.max(float(rank) * 1.5)
        a2a = c.alltoallv([_a2a_part(rank, d) for d in range(world)])
        assert [x.tobytes() for x in a2a] == [_a2a_part(s, rank).tobytes() for s in range(world)]
        c.barrier()
        q.put((rank, counts.tolist(), allb.tobytes(), m, c.backend))
    finally:
        c.close()


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_rccl_allgather_multi_rank(world):
    """Multi-rank RCCL (one process per GPU): counts all-gather, padded byte all-gather over xGMI and the
    compaction of every rank's slice.  Needs `world` visible GPUs; skipped on a smaller box."""
    from mandalorion_amd import _lib

    if _lib.device_count() < world:
        pytest.skip(f"{world} GPUs needed for {world} RCCL ranks")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_rccl_rank, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = sorted(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    sizes = [0 if r == 1 else r * 70001 + 13 for r in range(world)]
    want = b"".join(((np.arange(sizes[r]) * (r + 3)) % 251).astype(np.uint8).tobytes() for r in range(world))
    for rank, counts, allb, m, backend in out:
        assert backend == "rccl"
        assert counts == sizes
        assert allb == want
        assert m == 1.5 * (world - 1)
