"""Rehearsal of an N-rank D-module run on one GPU: the ranks run one after another in
this process, each on its own share of the LPT plan, exactly as define_isoforms runs them under a real
communicator -- except the transport, an in-process stand-in.

* placement reassembly (the default): allgather_bytes / alltoallv call c returns every rank's latest
  contribution to call c.  Four passes over the ranks: the first warms each rank's share (its own process
  in a real run: files cached, device buffers sized) and completes the count exchange, the second the size
  exchanges, the third the range placement's pieces, the fourth is timed and its placed files are checked
  against the one-rank run.
* gather reassembly (MANDO_REASSEMBLY=gather): ranks 1..N-1 hand their compacted payload to a recording
  stand-in for mando_gather_bytes, and rank 0 receives those bytes from it, then merges and writes.

The predicted N-GPU step = max over ranks of the rank's own step (+ rank 0's gather-side work and the
estimated RCCL transfer for gather).  Placement: the ranks' FASTA blocks go into one file at the same
time in a real run, and buffered writes to one file serialise in the kernel, so the prediction also
reports the step with every rank's FASTA placement serialised (an upper bound).

With PLACE_DUMP=<dir> a fourth, untimed pass saves each rank's placement blocks there (real sizes and
offsets of the N-rank plan), for tools/place_contention.py to place from N processes at once.

usage: python tools/rank_rehearsal.py <data dir with tmp_SS> N [threads]
"""
from __future__ import annotations

import hashlib
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


class _Place:
    """Placement stand-in: call c of allgather_bytes returns every rank's latest contribution to call c.
    Its early passes deliver incomplete pieces, which define._place drops for a `standin` transport."""

    standin = True

    def __init__(self, rank, world, store):
        self.rank, self.world, self.store, self.calls = rank, world, store, 0

    def allgather_bytes(self, blob):
        c = self.store.setdefault(self.calls, {})
        self.calls += 1
        c[self.rank] = np.array(blob, dtype=np.uint8, copy=True)
        empty = np.zeros(1, np.int64).view(np.uint8)
        parts = [c.get(r, empty) for r in range(self.world)]
        return np.concatenate(parts), np.array([p.size for p in parts], dtype=np.int64)

    def alltoallv(self, parts):
        """call c returns, by rank, each rank's latest part addressed to this one for call c"""
        c = self.store.setdefault(("a2a", self.calls), {})
        self.calls += 1
        c[self.rank] = [np.array(p, dtype=np.uint8, copy=True).ravel() for p in parts]
        return [c[r][self.rank] if r in c else np.zeros(0, np.uint8) for r in range(self.world)]

    def barrier(self):
        pass


class _Recorder:
    """A rank r != 0: its gather_bytes call hands the blob to the shared store and returns nothing."""

    def __init__(self, rank, world, store):
        self.rank, self.world, self.store = rank, world, store

    def gather_bytes(self, blob):
        self.store[self.rank] = np.array(blob, dtype=np.uint8, copy=True)
        return None, None


class _Root:
    """Rank 0: receives every recorded blob (its own first), as mando_gather_bytes would on the writer."""

    def __init__(self, world, store):
        self.rank, self.world, self.store = 0, world, store

    def gather_bytes(self, blob):
        self.store[0] = np.array(blob, dtype=np.uint8, copy=True)
        parts = [self.store[r] for r in range(self.world)]
        return np.concatenate(parts), np.array([p.size for p in parts], dtype=np.int64)


def sha(p):
    h = hashlib.sha256()
    with open(p, "rb") as fh:
        for b in iter(lambda: fh.read(1 << 24), b""):
            h.update(b)
    return h.hexdigest()


def _span(st, name):
    return sum(b - a for n, a, b in st["timeline"] if n == name)


def _dump_place(define, dump: str, cur: list):
    """Wraps define._place so that the dump pass saves every rank's real blocks (the buffer, per-root
    source offsets, roots, sizes and the all-rank size table) for tools/place_contention.py."""
    inner = define._place

    def place(path, buf, src, roots, sizes, g_sizes, comm, threads=0):
        if cur[0] is not None:
            np.savez(os.path.join(dump, f"r{cur[0]}_{os.path.basename(path)}.npz"), buf=buf, src=src,
                     roots=roots, sizes=sizes, g_sizes=g_sizes)
        return inner(path, buf, src, roots, sizes, g_sizes, comm, threads)

    define._place = place


def main_place(d, n, threads, ref, files):
    from mandalorion_amd import define

    store: dict = {}
    cur = [None]
    dump = os.environ.get("PLACE_DUMP")
    if dump:
        os.makedirs(dump, exist_ok=True)
        _dump_place(define, dump, cur)
    out = {"ranks": n, "reassembly": "place", "threads": threads, "rank_s": {}, "rank_phases_s": {}}
    for p in range(5 if dump else 4):  # the dump pass comes after the timed one
        for r in range(n):
            cur[0] = r if p == 4 else None
            t0 = time.perf_counter()
            st = define.define_isoforms(d, threads=threads, comm=_Place(r, n, store))
            print(f"[rehearsal] pass {p} rank {r}: {time.perf_counter() - t0:.2f} s", file=sys.stderr, flush=True)
            if p == 3:
                out["rank_s"][r] = round(time.perf_counter() - t0, 4)
                ph = {k: round(st[k], 4) for k in ("t_ingest", "t_cluster", "t_orient", "t_poa", "t_merge", "t_total")}
                ph["place_r2i"] = round(_span(st, "write_r2i"), 4)     # overlapped with the POA
                ph["place_fasta"] = round(_span(st, "write"), 4)      # after it, ends with the barrier
                out["rank_phases_s"][r] = ph
    got = {f: sha(os.path.join(d, f)) for f in files}
    out["reassembled_equals_one_rank"] = (got == ref) if ref else None
    out["reassembled_sha256"] = got
    out["predicted_step_s"] = round(max(out["rank_s"].values()), 4)
    pf = [v["place_fasta"] for v in out["rank_phases_s"].values()]
    out["predicted_step_serial_fasta_s"] = round(max(v - f for v, f in zip(out["rank_s"].values(), pf)) + sum(pf), 4)
    print(json.dumps(out), flush=True)


def main():
    from mandalorion_amd import define

    d, n = sys.argv[1], int(sys.argv[2])
    threads = int(sys.argv[3]) if len(sys.argv) > 3 else 16
    files = ("Isoform_Consensi.fasta", "reads2isoforms.txt")
    ref = {f: sha(os.path.join(d, f)) for f in files} if all(os.path.exists(os.path.join(d, f)) for f in files) else None
    if define._REASSEMBLY == "place":
        return main_place(d, n, threads, ref, files)
    store: dict = {}
    out = {"ranks": n, "rank_s": {}, "payload_bytes": {}}
    for r in list(range(1, n)) + [0]:
        comm = _Root(n, store) if r == 0 else _Recorder(r, n, store)
        # each rank's warmup step (its own process in a real run: files cached, device buffers sized for
        # its share), then the timed step
        define.define_isoforms(d, threads=threads, share=(r, n))
        t0 = time.perf_counter()
        st = define.define_isoforms(d, threads=threads, comm=comm)
        out["rank_s"][r] = round(time.perf_counter() - t0, 4)
        if r:
            out["payload_bytes"][r] = int(store[r].size)
        else:
            out["payload_bytes"][0] = int(store[0].size)
            out["rank0_phases_s"] = {k: round(st[k], 4) for k in ("t_ingest", "t_cluster", "t_orient", "t_poa",
                                                                   "t_merge", "t_write", "t_total")}
            out["rank0_compute_s"] = round(st["t_total"] - st["t_merge"] - st["t_write"], 4)
    got = {f: sha(os.path.join(d, f)) for f in files}
    out["reassembled_equals_one_rank"] = (got == ref) if ref else None
    out["reassembled_sha256"] = got
    # predicted N-GPU step: the slowest rank's own work, then rank 0's merge + write of everything, plus
    # the transfer of the other ranks' payloads into rank 0 (RCCL p2p over xGMI, estimated at 50 GB/s)
    others = max(v for r, v in out["rank_s"].items() if r != 0) if n > 1 else 0.0
    xfer = sum(v for r, v in out["payload_bytes"].items() if r != 0) / 50e9
    out["predicted_step_s"] = round(max(others, out["rank0_compute_s"]) + out["rank0_phases_s"]["t_merge"]
                                    + out["rank0_phases_s"]["t_write"] + xfer, 4)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
