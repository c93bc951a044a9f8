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
        c.barrier()


def _rccl_rank(rank, world, port, q):
    import os

    os.environ.update(WORLD_SIZE=str(world), RANK=str(rank), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    from mandalorion_amd.comm import Comm

    c = Comm.from_env(device=rank)
    try:
        # ragged sizes (rank 1 sends nothing): the padded ncclAllGather + per-slice compaction
        blob = ((np.arange(rank * 70001 + 13) * (rank + 3)) % 251).astype(np.uint8) if rank != 1 else np.zeros(0, np.uint8)
        allb, counts = c.allgather_bytes(blob)
        # the writer's gather: point-to-point sends to rank 0 (ragged, one empty)
        g, gc = c.gather_bytes(blob)
        assert gc.tolist() == counts.tolist()
        assert (g is None) == (rank != 0) and (g is None or g.tobytes() == allb.tobytes())
        m = c.max(float(rank) * 1.5)
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
