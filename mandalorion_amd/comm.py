"""Reassembly transport of the sharded D module (libmando `mando_comm_*`, include/mando.h).

One process per GPU, started by any launcher that exports WORLD_SIZE / RANK / LOCAL_RANK / MASTER_ADDR /
MASTER_PORT (the driver's elastic launcher does); the launcher only provides the environment.  Ranks rendezvous over a TCP
star on MASTER_ADDR:(MASTER_PORT + 1) (MANDO_COMM_PORT overrides; the launcher's own store holds
MASTER_PORT) and, when bound to a device context, exchange bytes over RCCL / xGMI.  The reference's
only cross-locus step is its Pool's ordered writer (defineIsoforms.py:130-166), which this replaces.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from . import _lib


class Comm:
    """A communicator of `world` ranks (rank 0 = the writer)."""

    def __init__(self, world: int, rank: int, addr: str = "127.0.0.1", port: int = 0, device_ctx=None,
                 timeout_s: float = 300.0):
        self.lib = _lib.load()
        self.world = int(world)
        self.rank = int(rank)
        h = ctypes.c_void_p()
        _lib.check(self.lib.mando_comm_init(device_ctx.handle if device_ctx is not None else None, self.world,
                                            self.rank, addr.encode(), int(port), float(timeout_s), ctypes.byref(h)))
        self.handle = h
        self.device_ctx = device_ctx

    @classmethod
    def from_env(cls, device: int | None = None, gpu: bool | None = None) -> "Comm":
        """From the launcher's environment; RCCL when a GPU is visible (gpu=None) or requested."""
        world = int(os.environ.get("WORLD_SIZE", "1"))
        rank = int(os.environ.get("RANK", "0"))
        addr = os.environ.get("MASTER_ADDR", "127.0.0.1")
        port = int(os.environ.get("MANDO_COMM_PORT", "0")) or int(os.environ.get("MASTER_PORT", "29500")) + 1
        if gpu is None:
            gpu = _lib.device_count() > 0
        ctx = None
        if gpu and world > 1:
            dev = int(os.environ.get("LOCAL_RANK", "0")) if device is None else device
            ctx = _lib.context(dev, slot=2)  # its own stream: the reassembly never queues behind a POA launch
        return cls(world, rank, addr, port, device_ctx=ctx)

    @property
    def backend(self) -> str:
        return "rccl" if self.lib.mando_comm_backend(self.handle) == 1 else "host"

    def allgather_counts(self, n: int) -> np.ndarray:
        out = np.zeros(self.world, dtype=np.int64)
        _lib.check(self.lib.mando_allgather_counts(self.handle, int(n), _lib.ptr(out)))
        return out

    def allgather_bytes(self, blob: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
        """Every rank's uint8 blob, concatenated in rank order, plus the per-rank counts."""
        blob = np.ascontiguousarray(blob, dtype=np.uint8)
        counts = self.allgather_counts(blob.size)
        out = np.empty(max(int(counts.sum()), 1), dtype=np.uint8)
        send = blob if blob.size else np.zeros(1, dtype=np.uint8)
        _lib.check(self.lib.mando_allgather_bytes(self.handle, _lib.ptr(send), int(blob.size), _lib.ptr(out),
                                                  _lib.ptr(counts)))
        return out[:int(counts.sum())], counts

    def gather_bytes(self, blob: np.ndarray) -> tuple[np.ndarray | None, np.ndarray]:
        """Every rank's uint8 blob, concatenated in rank order, on rank 0 (None elsewhere), plus the counts."""
        blob = np.ascontiguousarray(blob, dtype=np.uint8)
        counts = self.allgather_counts(blob.size)
        out = np.empty(max(int(counts.sum()), 1), dtype=np.uint8) if self.rank == 0 else None
        send = blob if blob.size else np.zeros(1, dtype=np.uint8)
        _lib.check(self.lib.mando_gather_bytes(self.handle, _lib.ptr(send), int(blob.size), _lib.ptr(out),
                                               _lib.ptr(counts)))
        return (out[:int(counts.sum())] if out is not None else None), counts

    def alltoallv(self, parts: list) -> list:
        """Personalised exchange: parts[r] (uint8) goes to rank r; returns, by rank, what every rank sent
        to this one.  The send counts are all-gathered first (each rank learns what it receives); the bytes
        go over RCCL point-to-point (mando_alltoallv_bytes), or over the host transport as one all-gather
        of every rank's parts of which each rank keeps its own."""
        parts = [np.ascontiguousarray(p, dtype=np.uint8).ravel() for p in parts]
        if len(parts) != self.world:
            raise ValueError("alltoallv: one part per rank")
        sc = np.array([p.size for p in parts], dtype=np.int64)
        allc, _ = self.allgather_bytes(sc.view(np.uint8))
        mat = allc.view(np.int64).reshape(self.world, self.world)
        rc = np.ascontiguousarray(mat[:, self.rank])
        roff = np.concatenate([[0], np.cumsum(rc)])
        send = np.concatenate(parts) if sc.sum() else np.zeros(1, dtype=np.uint8)
        if self.backend == "rccl" or self.world == 1:
            recv = np.empty(max(int(rc.sum()), 1), dtype=np.uint8)
            _lib.check(self.lib.mando_alltoallv_bytes(self.handle, _lib.ptr(send), _lib.ptr(sc), _lib.ptr(recv),
                                                      _lib.ptr(rc)))
            return [recv[roff[r]:roff[r + 1]] for r in range(self.world)]
        allb, cnt = self.allgather_bytes(send[:int(sc.sum())])
        base = np.concatenate([[0], np.cumsum(cnt)])
        out = []
        for r in range(self.world):
            a = int(base[r] + mat[r, :self.rank].sum())
            out.append(allb[a:a + int(mat[r, self.rank])])
        return out

    def max(self, v: float) -> float:
        x = ctypes.c_double(float(v))
        _lib.check(self.lib.mando_allreduce_max_f64(self.handle, ctypes.byref(x)))
        return x.value

    def barrier(self) -> None:
        _lib.check(self.lib.mando_comm_barrier(self.handle))

    def close(self) -> None:
        if getattr(self, "handle", None):
            self.lib.mando_comm_destroy(self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
