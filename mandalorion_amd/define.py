"""D module driver: the MI355X-native `defineIsoforms.py` (Mando.py -M D).

Same CLI and outputs as /root/reference/defineIsoforms.py:20-52 (`-i -p -c -g -w -m -W -n -j -u -d -a`);
writes <p>/Isoform_Consensi.fasta, <p>/reads2isoforms.txt and <p>/polyAWhiteList.bed.

Instead of one forked process per locus calling mappy + an `abpoa` subprocess per isoform
(defineIsoforms.py:130-153, SpliceDefineConsensus.py:876-931), the whole locus set goes through:
  1. clustering (libmando `mando_cluster_loci`: host threads read the files into HBM, HIP kernels
     cluster one locus per wave): peaks, isoform groups, RNG replay of every locus' draws and the
     determine_consensus subsample;
  2. orientation of every subsampled read against its isoform's first subsampled read
     (`mando_orient_segments`, HIP; the reads are gathered from the locus text already in HBM);
  3. the reference's per-isoform assembly logic (duplicate-primary rebinding, <=2 fallback, median
     length -> `-S`) on the host, on arrays;
  4. one batched POA consensus over all remaining isoforms (`mando_poa_segments`, HIP, reads again
     gathered from the device text);
  5. the ordered writer (sorted roots x IsoDict order, `Isoform{k}_{n}`).
The host-packed entry points (`mando_orient_batch`, `mando_poa_batch`) serve callers holding reads in
host memory (the abpoa-argv CLI, tests).
Loci shard across ranks (one process per GPU, mandalorion_amd.comm); the only exchange is one all-gather
of per-locus results to rank 0 for the writer (RCCL over xGMI).
"""
from __future__ import annotations

import argparse
import ctypes
import os
import sys
import threading
import time
from typing import Callable, Sequence

import numpy as np

from . import _lib, cluster, gtf

# mappy.revcomp's complement table (minimap2 seq_comp_table; csrc/revcomp.h): IUPAC, either case
COMP = bytes.maketrans(b"ACGTURYKMBVDHSWNacgturykmbvdhswn", b"TGCAAYRMKVBHDSWNtgcaayrmkvbhdswn")


def revcomp(s: str) -> str:
    """mappy.revcomp."""
    return s.encode().translate(COMP)[::-1].decode()


def gpu_orient(seqs, seq_off, grp_off, device: int = 0, max_hits: int = 4):
    """Per read: the strands (+1/-1) of its primary hits against its group's first read (HIP).  A read
    with more than max_hits primaries (n_hits == max_hits + 1) re-runs the batch with room for 8; more
    than 8 is refused rather than silently truncated."""
    from . import orient

    hits, nh = orient.orient_packed(seqs, seq_off, grp_off, device=device, max_hits=max_hits, slot=1)
    if len(nh) and int(nh.max()) > max_hits:
        if max_hits >= 8:
            raise _lib.MandoError(-5, "a read has more than 8 primary hits against its isoform's first read")
        return gpu_orient(seqs, seq_off, grp_off, device=device, max_hits=8)
    return hits, nh


def gpu_orient_segments(res, off, length, grp_off, device: int = 0, max_hits: int = 4):
    """gpu_orient over reads that stay in the clustering result's device text (no host packing)."""
    from . import orient

    d, n = res.device_text()
    hits, nh = orient.orient_segments(d, n, off, length, grp_off, device=device, max_hits=max_hits, slot=1)
    if len(nh) and int(nh.max()) > max_hits:
        if max_hits >= 8:
            raise _lib.MandoError(-5, "a read has more than 8 primary hits against its isoform's first read")
        return gpu_orient_segments(res, off, length, grp_off, device=device, max_hits=8)
    return hits, nh


def gpu_consensus(seqs, seq_off, grp_off, seeding, device: int = 0, info: dict | None = None, slot: int = 0):
    from . import poa

    return poa.poa_consensus_packed(seqs, seq_off, grp_off, seeding=seeding, device=device, info=info, slot=slot)


def usable_cores() -> int:
    """The host CPUs this process may use: its affinity, capped by the cgroup's CPU quota (cpu.max);
    os.cpu_count() is the whole machine, on a GPU box many times this process's share."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(q) // int(per)))
    except (OSError, ValueError):
        pass
    return max(1, n)


def _roots(out_tmp: str, sizes: dict | None = None, size_array: list | None = None) -> list[str]:
    """Locus roots of tmp_SS (defineIsoforms.py:130-139); sizes (optional) receives each root's
    <root>.psl size from the same directory scan, size_array (a list, optional) one int64 array of them
    aligned with the roots (0: no exact <root>.psl entry) -- no per-root dictionary work on 200,000 loci.
    The scan, the stat calls and the sort run natively (mando_list_roots); a root whose start field is
    not a plain decimal takes the Python path below, which parses (or raises) exactly as the reference
    does."""
    lib = _lib.load()
    # room for 512k roots in the first call (a second call repeats the whole scan: 200,000 loci took
    # two, 0.5 s per rank, r04g)
    cap_n, cap_b = 1 << 19, 1 << 24
    for _ in range(2):
        names = ctypes.create_string_buffer(cap_b)
        sz = np.empty(cap_n, dtype=np.int64)
        nr, nb = ctypes.c_int64(), ctypes.c_int64()
        rc = lib.mando_list_roots(out_tmp.encode(), 0, names, cap_b, _lib.ptr(sz), cap_n, ctypes.byref(nr),
                                  ctypes.byref(nb))
        if rc == -4:  # MANDO_E_CAP: the sizes are returned
            cap_n, cap_b = max(1, nr.value), max(1, nb.value)
            continue
        if rc != 0:
            break
        roots = names.raw[:nb.value].decode("utf-8", "surrogateescape").split("\0")[:-1]
        if sizes is not None:
            sizes.update((r, v) for r, v in zip(roots, sz[:nr.value].tolist()) if v >= 0)
        if size_array is not None:
            size_array.append(np.maximum(sz[:nr.value], 0))
        return roots
    d: dict = {}
    roots = _roots_py(out_tmp, d)
    if sizes is not None:
        sizes.update(d)
    if size_array is not None:
        size_array.append(np.array([d.get(r, 0) for r in roots], dtype=np.int64))
    return roots


def _roots_py(out_tmp: str, sizes: dict | None = None) -> list[str]:
    roots = set()
    with os.scandir(out_tmp) as it:
        for e in it:
            if ".psl" in e.name and e.is_file():
                r = e.name.split(".psl")[0]  # chrom~start~end (a '~' in a chrom breaks the reference too)
                roots.add(r)
                if sizes is not None and e.name == r + ".psl":
                    sizes[r] = e.stat().st_size
    return sorted(roots, key=lambda x: (x.split("~")[0], int(x.split("~")[1])))


def _root_names(out_tmp: str) -> list[str]:
    """The roots of _roots without their sizes: one directory read (mando_list_root_names; readdir's
    entry type decides, only symlinks and entries of unknown type are stat'ed)."""
    lib = _lib.load()
    cap_b = 1 << 24
    for _ in range(2):
        names = ctypes.create_string_buffer(cap_b)
        nr, nb = ctypes.c_int64(), ctypes.c_int64()
        rc = lib.mando_list_root_names(out_tmp.encode(), names, cap_b, ctypes.byref(nr), ctypes.byref(nb))
        if rc == -4:  # MANDO_E_CAP: the size is returned
            cap_b = max(1, nb.value)
            continue
        if rc != 0:
            break
        return names.raw[:nb.value].decode("utf-8", "surrogateescape").split("\0")[:-1]
    return _roots_py(out_tmp)


def _root_sizes(out_tmp: str, roots: list[str]) -> np.ndarray:
    """Size of each <root>.psl (0 when it is not a regular file), as _roots' size_array."""
    sizes = np.zeros(len(roots), dtype=np.int64)
    if roots:
        blob = ("\0".join(roots) + "\0").encode("utf-8", "surrogateescape")
        _lib.check(_lib.load().mando_root_sizes(out_tmp.encode(), blob, len(roots), 0, _lib.ptr(sizes)))
    return np.maximum(sizes, 0)


def _shared_roots(out_tmp: str, comm) -> tuple[list[str], np.ndarray]:
    """The root list and sizes on every rank: rank 0 reads the directory and all-gathers the names (the
    other ranks send nothing), then every rank stats the <root>.psl files of its slice of the list and a
    second all-gather assembles the sizes.  Rank 0 stat'ing all 200,000 files itself took 0.13-0.30 s
    of every rank's step at 8 ranks (rank 0's ingest in the r04f2 rehearsal, the other ranks 0.03 s).
    A slice that arrives with the wrong length (only under the rehearsal's in-process stand-in, whose
    later ranks have not run yet) is stat'ed here instead: the sizes drive both the shard plan and the
    chunk plan's HBM budget, so none may be missing."""
    err = None
    if comm.rank == 0:
        try:
            roots = _root_names(out_tmp)
            names = "\0".join(roots).encode("utf-8", "surrogateescape")
            blob = np.concatenate([np.array([len(roots), len(names)], np.int64).view(np.uint8),
                                   np.frombuffer(names, np.uint8)])
        except Exception as e:  # the other ranks learn of it (n = -1) instead of waiting for a list
            err = e
            blob = np.array([-1, 0], np.int64).view(np.uint8)
    else:
        blob = np.zeros(0, np.uint8)
    allb, counts = comm.allgather_bytes(blob)
    if err is not None:
        raise err
    if comm.rank != 0:
        part = allb[:int(counts[0])]
        n, nb = (int(x) for x in part[:16].view(np.int64))
        if n < 0:
            raise RuntimeError("rank 0 could not list the locus roots (its error is the first one raised)")
        names = part[16:16 + nb].tobytes().decode("utf-8", "surrogateescape")
        roots = names.split("\0") if n else []
    n, world = len(roots), comm.world
    cut = [n * r // world for r in range(world + 1)]
    mine = _root_sizes(out_tmp, roots[cut[comm.rank]:cut[comm.rank + 1]])
    allb, counts = comm.allgather_bytes(mine.view(np.uint8))
    sizes = np.zeros(n, dtype=np.int64)
    off = np.concatenate([[0], np.cumsum(counts)])
    for r in range(world):
        if int(counts[r]) == 8 * (cut[r + 1] - cut[r]):
            sizes[cut[r]:cut[r + 1]] = allb[int(off[r]):int(off[r + 1])].view(np.int64)
        else:
            sizes[cut[r]:cut[r + 1]] = _root_sizes(out_tmp, roots[cut[r]:cut[r + 1]])
    return roots, sizes


def _size_costs(sizes: np.ndarray) -> np.ndarray:
    """Per-locus POA cost estimate for the shard plan, from the file sizes the root scan returns (no
    per-file I/O): a locus of n reads of length L costs ~n L^2 (n L (2w+1) 1.1 L) and
    its file holds ~n L bytes, so with the read count bounded by the subsample the cost grows as the
    size squared.  Reading each file's first record instead (round 3) took 1 s per rank per step on
    20,000 loci and 8-9 s on 200,000 (r04f), on the critical path of every rank."""
    sz = np.asarray(sizes, dtype=np.float64)
    return sz * sz


def _lpt_owner(cost: np.ndarray, world: int, head: int = 64) -> np.ndarray:
    """The shard plan (every rank computes the same one): loci by cost, descending; the heaviest
    head x world go to the least-loaded rank one at a time (LPT: they set the launches' floors), the
    rest in a snake over the ranks ordered by load.  Vectorised: a Python argmin per locus took 0.4-0.8 s
    for 200,000 loci on every rank (r04).  (Contiguous root ranges per rank after the head balanced the
    POA worse in the round-4 rehearsal -- 8 ranks: POA 1.42-1.69 s against 1.44-1.52 s -- and were
    dropped.)"""
    import heapq

    order = np.argsort(-cost, kind="stable")
    owner = np.empty(len(cost), dtype=np.int64)
    k = min(len(order), head * world)
    h = [(0.0, r) for r in range(world)]
    for i in order[:k].tolist():
        ld, r = h[0]
        owner[i] = r
        heapq.heapreplace(h, (ld + float(cost[i]), r))
    rest = order[k:]
    if len(rest):
        by_load = np.array([r for _, r in sorted(h)], dtype=np.int64)
        m = np.arange(len(rest)) % (2 * world)
        owner[rest] = by_load[np.where(m < world, m, 2 * world - 1 - m)]
    return owner


class Assembly:
    """determine_consensus (SpliceDefineConsensus.py:876-931) minus the POA call, for every isoform at
    once, on arrays.  Emissions: every primary hit of a subsampled read writes the read once, in hit
    order, re-bound by the hits before it (SDC:902-907); the isoform's sequences are its emissions."""

    def __init__(self, res: cluster.ClusterResult, hits: np.ndarray, n_hits: np.ndarray):
        sub_off = res.sub_off
        n_iso = len(sub_off) - 1
        n_sub = int(sub_off[-1])
        hits = np.asarray(hits).reshape(n_sub, -1) if n_sub else np.zeros((0, 1), np.int8)
        H = hits.shape[1]
        nh = np.asarray(n_hits)[:n_sub]
        if len(nh) and int(nh.max()) > H:
            # the orientation reports max_hits + 1 for a read with more primary hits than it kept: the
            # caller must re-run such reads with room for all of them (gpu_orient* do)
            bad = int(np.argmax(nh > H))
            raise ValueError(f"subsampled read {bad}: {int(nh[bad])} hits reported for {H} hit columns "
                             "(orientation overflow not re-run)")
        self.e_read = np.repeat(np.arange(n_sub), nh)            # emission -> subsample slot
        # emission j of a read is its hit j, re-bound by the hits before it: the running product of the
        # read's hit strands (+1 / -1) up to j.  Most reads have one hit, so the product starts from
        # column 0 and only the emissions at column >= c take column c (entries past a read's hit count
        # are never read: the kernel does not write them)
        first = np.cumsum(nh) - nh
        e_col = np.arange(len(self.e_read)) - np.repeat(first, nh)
        e_sign = hits[self.e_read, 0] if len(self.e_read) else np.zeros(0, np.int8)
        for c in range(1, H):
            m = np.nonzero(e_col >= c)[0]
            if not len(m):
                break
            e_sign[m] = e_sign[m] * hits[self.e_read[m], c]
        self.e_sign = e_sign                                      # row-major = hit order per read
        iso_of_sub = np.repeat(np.arange(n_iso), np.diff(sub_off))
        self.e_iso = iso_of_sub[self.e_read] if n_sub else np.zeros(0, np.int64)
        self.n_emit = np.bincount(self.e_iso, minlength=n_iso) if n_iso else np.zeros(0, np.int64)
        empty = np.nonzero(self.n_emit == 0)[0]
        if len(empty):
            raise IndexError(f"isoform {int(empty[0])}: no subsampled read maps to the first one "
                             "(the reference raises IndexError at SpliceDefineConsensus.py:912)")
        self.first_emit = np.searchsorted(self.e_iso, np.arange(n_iso))
        self.direct = self.n_emit <= 2
        self.poa_iso = np.nonzero(~self.direct)[0]
        self.e_rec = res.sub[self.e_read] if n_sub else np.zeros(0, np.int64)
        # -S when the median subsample length (all subsampled reads, mapped or not) is >= 8000
        # (np.median of a group = mean of its two middle values: sort inside groups, pick them)
        self.seeding = np.zeros(len(self.poa_iso), dtype=np.uint8)
        # (no read of 8,000 or more anywhere: no median can reach it)
        if len(self.poa_iso) and len(res.seq_len) and int(res.seq_len.max()) >= 8000:
            lens = res.seq_len[res.sub].astype(np.int64)
            m = np.diff(sub_off)
            # the median can reach 8000 only when the upper middle value does, i.e. when at least
            # ceil(m/2) of the group's reads are >= 8000; only those groups are sorted
            n8k = (np.add.reduceat((lens >= 8000).astype(np.int64), np.minimum(sub_off[:-1], n_sub - 1)) if n_sub
                   else np.zeros(n_iso, np.int64))
            n8k = np.where(m > 0, n8k, 0)
            cand = np.zeros(n_iso, dtype=bool)
            cand[self.poa_iso] = True
            cand &= n8k >= m - m // 2
            if cand.any():
                gid = np.repeat(np.arange(n_iso), m)
                keep = cand[gid]
                srt = np.sort((gid[keep].astype(np.int64) << 32) | lens[keep]) & 0xffffffff  # sorted inside groups
                co = np.zeros(n_iso + 1, dtype=np.int64)
                np.cumsum(np.where(cand, m, 0), out=co[1:])
                ci = np.nonzero(cand)[0]
                med2 = np.zeros(n_iso, dtype=np.int64)
                med2[ci] = srt[co[ci] + (m[ci] - 1) // 2] + srt[co[ci] + m[ci] // 2]
                self.seeding = (med2[self.poa_iso] >= 16000).astype(np.uint8)
        self.res = res

    def poa_segments(self):
        """The POA input as (text offset, length, reverse-complement flag) per emission + group offsets."""
        sel = ~self.direct[self.e_iso]
        rec = self.e_rec[sel]
        grp = np.zeros(len(self.poa_iso) + 1, dtype=np.int64)
        np.cumsum(self.n_emit[self.poa_iso], out=grp[1:])
        return self.res.seq_off[rec], self.res.seq_len[rec], (self.e_sign[sel] == -1).astype(np.int8), grp

    def poa_input(self):
        """The POA input packed on the host (for an injected consensus_fn)."""
        off, length, rc, grp = self.poa_segments()
        seqs, so = _lib.pack_segments([self.res.text], off, length, rc=rc)
        return seqs, so, grp


# inputs of more than _TWO_CHUNK_BYTES of locus text run in chunks of at most this many bytes: a 4 GiB chunk's
# text, clustering scratch and gathered reads (about 7x the text, three chunks in flight) leave room for
# both POA launch kinds' one-group grids in a 288 GB HBM (config 4 on one GPU; r04e: 8 GiB chunks left
# the narrow launch 3,440 of its 3,840 slots, a persistent grid that held the CUs the next chunk's
# orientation waited for)
_CHUNK_BYTES = int(os.environ.get("MANDO_CHUNK_BYTES", str(4 << 30)))
# inputs of at least _BIG_INPUT_BYTES (config 4 on one or two GPUs: 62 / 31 GB) run in 6 GiB chunks unless
# MANDO_CHUNK_BYTES is set: config 4 14.2-14.4 s per step against 14.7 s with 4 GiB (5 / 7 GiB 14.4-14.6 s),
# rank 0's 2-rank share 7.24-7.32 against 7.55-7.56 s; rank 0's 4-rank share (15.5 GB) had one 1 s slower
# step in each 6 GiB run and keeps 4 GiB (profiles/r04cb_chunk_bytes_ab.txt)
_BIG_INPUT_BYTES = 24 << 30
_BIG_CHUNK_BYTES = _CHUNK_BYTES if "MANDO_CHUNK_BYTES" in os.environ else 6 << 30
# inputs with at least this much locus text run in two chunks (or more, past _CHUNK_BYTES); 10,000
# config-3 loci are 3.1 GB, 20,000 are 6.2 GB.  At 20,000 loci one chunk and two have the same mean step
# (1.78 / 1.77 s over 24 steps each), but two chunks put chunk 2's clustering and orientation kernels
# beside chunk 1's POA, and in about one step in four the wide POA launch then runs 3x slower (POA
# kernels 1.61-1.67 s against 1.32 s); one chunk has no such step (1,245-1,251 ms in all 24), so inputs
# below one byte-capped chunk run in one (r03 onechunk)
_TWO_CHUNK_BYTES = 8 << 30
# fewer loci than this always run in one chunk (a few large loci: SIRV-like, config 5)
_MIN_LOCI_CHUNKED = 1024
# the first chunk of a many-chunk plan, as a share of one chunk: small, so the first POA launch starts
# early, large enough to fill the chip (config 4: 0.4 against 0.6 / 0.75 in r07f; MANDO_FIRST_FRAC is the
# A/B knob)
_FIRST_FRAC = float(os.environ.get("MANDO_FIRST_FRAC", "0.4"))
def _chunk_plan(text_bytes: int, n_loci: int, n_chunks: int = 0,
                fracs: list | None = None) -> tuple[int, list | None]:
    """(chunks, cumulative byte fractions of the cuts or None for equal chunks).  n_chunks > 0 (or
    MANDO_CHUNKS) forces the count; a two-chunk plan cuts at 0.3 of the bytes unless `fracs` (cumulative
    fractions of the cuts, any count) is given."""
    if fracs:
        return max(1, min(len(fracs) + 1, max(1, n_loci))), list(fracs)
    if n_chunks <= 0 and os.environ.get("MANDO_CHUNKS"):
        n_chunks = int(os.environ["MANDO_CHUNKS"])
    if n_chunks <= 0:
        if text_bytes < _TWO_CHUNK_BYTES or n_loci < _MIN_LOCI_CHUNKED:
            n_chunks = 1
        else:
            k = -(-text_bytes // (_BIG_CHUNK_BYTES if text_bytes >= _BIG_INPUT_BYTES else _CHUNK_BYTES))
            if k > 1:
                fracs = [(_FIRST_FRAC + i) / k for i in range(k)]
                n_chunks = k + 1
            else:
                n_chunks = 2
    if n_chunks == 2 and fracs is None:
        fracs = [0.3]
    return max(1, min(n_chunks, max(1, n_loci))), fracs


# HBM plan of one call (bytes per byte of a chunk's locus text, measured on config-4 chunks with
# MANDO_WS_LOG=1: profiles/r04c_config4_ws_log.txt): the device text itself (pool buffers rounded to
# 256 MB: the chunks in flight -- clustering k+1, POA k, writing k-1 -- plus one cached), the clustering
# scratch of the largest chunk (K1 records and cs runs 2.56x the text, K2 maps and outputs 1.98x; one set
# per call, reused, allocated with 1/4 headroom) and the reads gathered for orientation and for the POA
# (0.42x each)
_HBM_USABLE = 0.92
# chunks whose buffers may be alive at once: clustering k+2 while k+1 waits for the POA, k runs it and
# k-1's wide part finishes and is written (the pool of locus-text buffers in poa_budget counts four)
_MAX_INFLIGHT = int(os.environ.get("MANDO_INFLIGHT", "4"))
# multi-rank reassembly: "place" -- the ranks exchange per-root isoform counts and byte sizes (two small
# all-gathers), send each block of their roots' output bytes to the rank that owns that range of the file
# (one personalised exchange per file) and each writes its own contiguous range of the shared output
# files; reads2isoforms.txt is placed while the POA runs (it needs only the clustering).  "gather" -- every rank's results go to rank
# 0 (one RCCL gather), which writes both files (ranks on nodes that share no output directory).
_REASSEMBLY = os.environ.get("MANDO_REASSEMBLY", "place")
_CLUSTER_SCRATCH_PER_TEXT = 1.25 * 4.55
_GATHERED_PER_TEXT = 0.42


def poa_budget(total_hbm: int, span_text: list) -> int:
    """Bytes the POA workspaces may take in a call whose chunks hold span_text bytes of locus text."""
    big = max(span_text) if span_text else 0
    pool = min(len(span_text), 4) * (big + (256 << 20))
    reserve = pool + int((_CLUSTER_SCRATCH_PER_TEXT + 2 * _GATHERED_PER_TEXT) * big) + (4 << 30)
    return max(4 << 30, int(_HBM_USABLE * total_hbm) - reserve)


# The wide groups of a chunk (bands over one 128-column chunk: the two-wave instantiation) run as a batch
# of their own on this context slot and a host thread of their own, beside the chunk's other groups: the
# next chunk's narrow launch then no longer waits for this chunk's wide one (a wide launch now and then
# takes twice its time).  Every group's consensus is the same either way: the library splits
# each batch by the same rule itself, so a group on the other side of the split here would only run in
# the other batch as its own kind.
_WIDE_SLOT = 5
_SPLIT_WIDE = os.environ.get("MANDO_SPLIT_WIDE", "1") != "0"
# the library's launch split (capi.hip poa_batch_impl): abPOA's adaptive band w = b + f * mean read
# length (float, truncated), wide when 2w + 1 exceeds one 128-column chunk's 116 usable columns
_BAND_B, _BAND_F, _WIDE_BAND = 10, np.float32(0.01), 116


def _wide_groups(length, grp_off, seeding) -> np.ndarray:
    n = np.diff(grp_off)
    cs = np.zeros(len(length) + 1, dtype=np.int64)
    np.cumsum(np.maximum(np.asarray(length, dtype=np.int64), 0), out=cs[1:])
    mean = (cs[grp_off[1:]] - cs[grp_off[:-1]]) // np.maximum(n, 1)
    w = _BAND_B + (_BAND_F * mean.astype(np.float32)).astype(np.int64)
    wide = 2 * w + 1 > _WIDE_BAND
    if seeding is not None:
        wide &= np.asarray(seeding) == 0
    return wide


class _Pending:
    """A part of a chunk's consensi still running on the wide context: a future of (cons, cons_off, info)
    and the part's group indices."""

    def __init__(self, fut, gidx):
        self.fut, self.gidx = fut, gidx

    def result(self):
        cons, cons_off, info = self.fut.result()
        return cons, cons_off, self.gidx, info


def _group_subset(off, length, rc, grp_off, seeding, mask):
    """The groups where mask holds, as (their indices, off, length, rc, grp_off, seeding) of a batch."""
    gidx = np.flatnonzero(mask)
    n = np.diff(grp_off)[gidx]
    starts = grp_off[:-1][gidx]
    g2 = np.zeros(len(gidx) + 1, dtype=np.int64)
    np.cumsum(n, out=g2[1:])
    ridx = np.repeat(starts - g2[:-1], n) + np.arange(int(g2[-1]), dtype=np.int64)
    sd = None if seeding is None else np.asarray(seeding)[gidx]
    return gidx, off[ridx], length[ridx], (None if rc is None else rc[ridx]), g2, sd


def define_isoforms(path: str, *args, device: int = 0, consensus_fn: Callable | None = None, **kw) -> dict:
    """Runs the D module on <path>/tmp_SS/*.psl (arguments: _define_isoforms).  The POA context's workspace
    budget is the call's own: it goes back to the library's default policy when the call returns, so a
    later direct POA call on the same context does not inherit this call's chunk plan."""
    try:
        return _define_isoforms(path, *args, device=device, consensus_fn=consensus_fn, **kw)
    finally:
        for slot in (0, _WIDE_SLOT):
            c = _lib._ctx_cache.get((device, slot)) if consensus_fn is None else None
            if c is not None and c.handle is not None:
                c.set_poa_budget(0)


def _define_isoforms(path: str, cutoff: float = 0.1, genome_file: str = "None", splice_site_width: int = 1,
                     minimum_read_count: int = 2, white_list_polyA: Sequence[str] = ("0",), threads: int = 0,
                     junctions: str = "gtag,gcag,atac,ctac,ctgc,gtat", upstream_buffer: int = 10,
                     downstream_buffer: int = 50, seed: int = 0, device: int = 0,
                     orient_fn: Callable | None = None, consensus_fn: Callable | None = None,
                     cluster_fn: Callable | None = None, comm=None, verbose: bool = False, n_chunks: int = 0,
                     share: tuple[int, int] | None = None, chunk_fracs: list | None = None) -> dict:
    """Runs the D module on <path>/tmp_SS/*.psl.  orient_fn(seqs, seq_off, grp_off) -> (hits, n_hits),
    consensus_fn(seqs, seq_off, grp_off, seeding) -> (cons bytes, cons_off) and cluster_fn (the signature
    of cluster.cluster_loci) default to the HIP path.
    comm (mandalorion_amd.comm.Comm, optional): shard the loci over comm.world ranks; rank 0 writes.
    share (r, N), without comm: run only rank r's loci of an N-rank plan, as one process writing its own
    files (the per-rank load of a multi-GPU run, measured on one GPU)."""
    t0 = time.perf_counter()
    rank, world = (comm.rank, comm.world) if comm is not None else (0, 1)
    plan_rank, plan_world = (rank, world) if share is None or comm is not None else share
    # the HIP path keeps the reads on the device (gathered from the clustering's device text); injected
    # host functions get them packed
    dev_orient = orient_fn is None
    dev_poa = consensus_fn is None
    poa_launches = []  # per POA call: DP cells, kernel ms, read + consensus bytes (the roofline's inputs)

    poa_slots: dict = {}
    slot_lock = threading.Lock()

    def _gpu_poa(res, off, length, rc, g, sd, slot=None, record=True):
        # one device context (stream + buffers) per POA host thread: slots 0 and 3 (1: orientation,
        # _WIDE_SLOT: the wide groups of a split chunk)
        from . import poa

        if slot is None:
            tid = threading.get_ident()
            with slot_lock:
                slot = poa_slots.setdefault(tid, 3 * len(poa_slots))
        info = {}
        d, n = res.device_text()
        out = poa.poa_consensus_segments(d, n, off, length, rc, g, seeding=sd, device=device, info=info, slot=slot)
        if "kernel_ms" in info:
            info["read_bytes"] = int(np.asarray(length, dtype=np.int64).sum())
            info["cons_bytes"] = int(out[1][-1])
            info["reads"] = int(g[-1])
            if record:
                poa_launches.append(info)
        return out + (info,)

    def run_poa(res, prep):
        """The chunk's consensi as parts [(cons, cons_off, group index or None), or _Pending]."""
        asm = prep[0]
        if not dev_poa:
            return [consensus_fn(*prep[1:], asm.seeding) + (None,)]
        off, length, rc, gro = prep[1:]
        if split_wide:
            wide = _wide_groups(length, gro, asm.seeding)
            if wide.any() and not wide.all():
                # the wide groups run as their own batch on their own context and thread, so that the
                # next chunk's narrow launch does not wait for this chunk's wide one
                sub = [_group_subset(off, length, rc, gro, asm.seeding, m) for m in (~wide, wide)]
                add("split_wide_groups", int(wide.sum()))
                fut = gpu_wide.submit(_gpu_poa, res, *sub[1][1:], slot=_WIDE_SLOT, record=False)
                a = _gpu_poa(res, *sub[0][1:], record=False)
                return [(a[0], a[1], sub[0][0], a[2]), _Pending(fut, sub[1][0])]
        a = _gpu_poa(res, off, length, rc, gro, asm.seeding)
        return [(a[0], a[1], None)]
    out_path = path + "/"
    out_tmp = out_path + "/tmp_SS"
    wl = list(white_list_polyA)
    left, right, poly = {}, {}, []
    if genome_file != "None" and (genome_file.endswith(".gtf.gz") or genome_file.endswith(".gtf")):
        _, left, right, poly = gtf.parse_genome(genome_file, wl)
    if rank == 0:
        gtf.write_polya_bed(out_path + "/polyAWhiteList.bed", poly, wl)
    if world > 1 and hasattr(comm, "allgather_bytes"):
        # one root scan (rank 0's, as the reference lists the roots once in its parent process,
        # defineIsoforms.py:130-139), shared with the other ranks: eight ranks stat-ing the same 200,000
        # files at once contend for the directory
        roots, root_sizes = _shared_roots(out_tmp, comm)
    else:
        size_arr: list = []
        roots = _roots(out_tmp, size_array=size_arr)
        root_sizes = size_arr[0]
    # shard loci over ranks: LPT on the DP-cost estimate of SURVEY.md §8(e), results regathered in root order
    mine = list(range(len(roots)))
    if plan_world > 1:
        owner = _lpt_owner(_size_costs(root_sizes), plan_world)
        mine = np.nonzero(owner == plan_rank)[0].tolist()
    my_roots = [roots[i] for i in mine]
    chroms = [r.split("~")[0] for r in my_roots]
    bidx = gtf.BoundsIndex(left, right)
    ann = ([bidx.bounds(r.split("~")[0], int(r.split("~")[1]), int(r.split("~")[2])) for r in my_roots]
           if bidx else None)
    t1 = time.perf_counter()
    timeline = [("ingest", 0.0, t1 - t0)]
    # Chunked pipeline: clustering of chunk k+1 (host C++ threads, GIL released) overlaps orientation +
    # POA of chunk k on the GPU.  Every POA launch lasts at least as long as its longest group, so few,
    # large launches are best:
    # * inputs above one byte-capped chunk (config 4 on one GPU: ~60 GB of locus text) run in contiguous
    #   chunks of at most _CHUNK_BYTES, the first 0.4 of one, so that its POA starts early;
    # * smaller inputs (config 3, a multi-GPU rank's share) and few loci (SIRV-like, config 5) run in
    #   one chunk.
    sizes = root_sizes[np.asarray(mine, dtype=np.int64)]
    n_chunks, fracs = _chunk_plan(int(sizes.sum()), len(my_roots), n_chunks, chunk_fracs)
    cuts = [0]
    if n_chunks > 1:
        cs = np.cumsum(sizes)
        fr = fracs or [k / n_chunks for k in range(1, n_chunks)]
        for f in fr:
            cuts.append(int(np.searchsorted(cs, cs[-1] * f)) + 1)
    cuts.append(len(my_roots))
    cuts = sorted(set(min(max(c, 0), len(my_roots)) for c in cuts))
    parts = [np.arange(cuts[k], cuts[k + 1]) for k in range(len(cuts) - 1) if cuts[k + 1] > cuts[k]]
    parts = parts or [np.arange(0)]
    # one rank: each chunk's part of both files is written as soon as it is done
    stream_out = world == 1
    placed = world > 1 and _REASSEMBLY == "place"
    names_parts: dict = {}
    mine_a = np.asarray(mine, dtype=np.int64)
    # the POA workspaces' HBM budget for this call, from the chunk plan (no free-memory query during the
    # call: the clustering thread allocates the next chunk's buffers while a POA launch sizes its
    # workspace).  The plan reserves this call's clustering buffers; buffers an earlier, larger call left
    # in the clustering's caches are freed first, or they would sit in HBM the plan counts as the POA's
    # (round 4: a rank-share call after a 6 GiB-chunk call asked for 176 GB of POA workspace that the
    # earlier call's caches still held, MANDO_E_NOMEM).
    pctx = None
    hbm = {}
    if dev_poa or cluster_fn is None:
        span_text = [int(sizes[ix].sum()) for ix in parts]
        big = max(span_text) if span_text else 0
        held = _lib.cache_trim(device, text_cap_max=big + (512 << 20),
                               scratch_max=int(1.25 * _CLUSTER_SCRATCH_PER_TEXT * big) + (1 << 30))
        hbm = {"cache_held_start": held}
    # one rank, several chunks: each chunk's wide groups run as a separate batch (_WIDE_SLOT)
    split_wide = dev_poa and world == 1 and len(parts) > 1 and _SPLIT_WIDE
    if dev_poa:
        pctx = _lib.context(device, 0)
        total_hbm = pctx.memory()[0]
        hbm.update(total=total_hbm, poa_budget=poa_budget(total_hbm, span_text))
        if split_wide:
            # the wide batches' context takes an eighth of the POA budget (their launches held 6-17 GB
            # of config 4's ~195 GB), the chunk's own context the rest
            wb = hbm["poa_budget"] // 8
            _lib.context(device, _WIDE_SLOT).set_poa_budget(wb)
            pctx.set_poa_budget(hbm["poa_budget"] - wb)
            hbm["wide_budget"] = wb
        else:
            pctx.set_poa_budget(hbm["poa_budget"])

    # with several chunks in flight, two cores stay with the GPU driver, assembly and compaction threads
    n_cpu = threads if threads > 0 else usable_cores()
    cl_threads = max(1, n_cpu - 2) if len(parts) > 1 and n_cpu > 4 else threads
    if world > 1:
        # several ranks on one node read their locus files at once, a CPU copy out of one page cache:
        # a rank's clustering reads with its share of the node's usable cores (at least 2).  On the
        # one-GPU box (a 16-core quota) 8 ranks x 2 readers read their real 8-rank config-4 shares in
        # 0.59 s (104 GB/s in all) and 8 x 16 in 1.16-1.40 s (48 GB/s: 128 threads on 16 cores;
        # profiles/r08a_read_contention_*)
        local_world = int(os.environ.get("LOCAL_WORLD_SIZE", "0")) or world
        cl_threads = min(cl_threads if cl_threads > 0 else n_cpu, max(2, usable_cores() // max(1, local_world)))

    # backpressure: at most _MAX_INFLIGHT chunks hold their buffers (locus text on host and device,
    # clustering results) at once -- clustering runs ahead of the POA otherwise, and a many-chunk input
    # (config 4 on one GPU; any input under the CPU restatements) would hold every chunk at once
    inflight = threading.BoundedSemaphore(_MAX_INFLIGHT)

    def run_cluster(k, ix):
        inflight.acquire()
        try:
            r = _run_cluster(ix)
        except BaseException:
            inflight.release()
            raise
        if placed:
            # the chunk's isoform order and member names, copied out: reads2isoforms.txt is placed from
            # them while the POA runs (the chunk's buffers go back to their pools after its POA)
            names_parts[k] = _compact_names(_names_payload(r[0], mine_a[ix]))
        return r

    def _run_cluster(ix):
        # clustering (host C++ threads, GIL released), then the orientation input: the subsampled reads
        tc = time.perf_counter()
        r = (cluster_fn or cluster.cluster_loci)(
            [os.path.join(out_tmp, my_roots[i] + ".psl") for i in ix], [chroms[i] for i in ix],
            ann=[ann[i] for i in ix] if ann else None,
            device=device, cutoff=cutoff, splice_site_width=splice_site_width,
            minimum_read_count=minimum_read_count, upstream_buffer=upstream_buffer,
            downstream_buffer=downstream_buffer, junctions=junctions, seed=seed, threads=cl_threads)
        te = time.perf_counter()
        timeline.append(("cluster", tc - t0, te - t0))
        bad = np.nonzero(r.locus_status != 0)[0]
        if len(bad):
            i = int(bad[0])
            code = int(r.locus_status[i])
            r.close()
            raise RuntimeError(f"locus {my_roots[ix[i]]}: {cluster.STATUS.get(code, code)} "
                               "(the reference's locus worker raises here)")
        r.on_close = inflight.release  # the chunk leaves the pipeline when its buffers are released
        if dev_orient and getattr(r, "orient_hits", None) is not None:
            o_in = (None, None)  # oriented inside the clustering call
        elif dev_orient:
            o_in = (r.seq_off[r.sub], r.seq_len[r.sub])
        else:
            o_in = _lib.pack_segments([r.text], r.seq_off[r.sub], r.seq_len[r.sub])
        return r, te - tc, o_in, time.perf_counter() - te

    from concurrent.futures import ThreadPoolExecutor

    stats = {"loci": len(roots), "isoforms": 0, "poa_groups": 0, "records": 0, "poa_reads": 0,
             "t_ingest": t1 - t0, "t_cluster": 0.0, "t_pack": 0.0, "t_orient": 0.0, "t_assemble": 0.0,
             "t_poa": 0.0, "chunks": len(parts), "poa_launches": poa_launches, "split_wide_groups": 0}
    payloads = []
    stats["timeline"] = timeline
    stats["hbm"] = hbm

    def assemble(res, hits, n_hits):
        ta = time.perf_counter()
        asm = Assembly(res, hits, n_hits)
        prep = (asm,) + tuple(asm.poa_segments() if dev_poa else asm.poa_input())
        te = time.perf_counter()
        add("t_assemble", te - ta)
        timeline.append(("assemble", ta - t0, te - t0))
        return prep

    # Staged pipeline over chunks: clustering (one host thread driving the C++ pool, chunks in order) ->
    # orientation (main thread, GPU slot 1) -> emission assembly (host thread) -> POA (one host thread,
    # GPU slot 0) -> writer.
    lock = threading.Lock()

    def add(key, v):
        with lock:
            stats[key] += v

    def poa_job(res, asm_fut, ix):
        prep = asm_fut.result()
        tp = time.perf_counter()
        pl = _poa_chunk(res, mine_a[ix], prep, run_poa, stats, lock, poa_launches)
        timeline.append(("poa", tp - t0, time.perf_counter() - t0))
        if world > 1:
            # several ranks: the chunk's results are gathered at the end, so its referenced bytes are
            # copied out now and its buffers (locus text on host and device) go back to their pools --
            # a many-chunk rank share holds only the chunks in flight
            del prep
            pl = _compact_cons(pl) if placed else _compact(pl)
            res.close()
        return pl, res

    # one POA host thread and device context (r02: a second context sized its workspace from the HBM the
    # first one left free -- a quarter of the slots, the persistent grid, 2.9 s, in 3 of 30 config-3 steps)
    with ThreadPoolExecutor(max_workers=1) as ex, ThreadPoolExecutor(max_workers=1) as host, \
            ThreadPoolExecutor(max_workers=1) as writer, \
            ThreadPoolExecutor(max_workers=1) as gpu_poa, ThreadPoolExecutor(max_workers=1) as gpu_wide:
        cl = [ex.submit(run_cluster, k, ix) for k, ix in enumerate(parts)]
        poa_futs = []
        # one rank: reads2isoforms.txt needs only the clustering, so each chunk's part of it is written
        # by the host thread (after the chunk's assembly) while the POA runs; the FASTA follows each POA
        fa = r2 = None
        r2_futs = []
        n_iso_before = 0
        if stream_out:
            fa = open(out_path + "/Isoform_Consensi.fasta", "wb")
            r2 = open(out_path + "/reads2isoforms.txt", "wb")

        fa_futs = []

        def write_fasta(poa_fut, counter0, r2_fut):
            # one rank: the writer thread appends each chunk's FASTA part as soon as its POA is done (in
            # chunk order: one thread, FIFO), off the main thread that orients the next chunk meanwhile;
            # once both of its parts are written the chunk's buffers (locus text on host and device)
            # go back to their pools, so a many-chunk run holds only the chunks in flight
            pl, res = poa_fut.result()
            if "_finish" in pl:  # the chunk's wide groups ran beside the next chunk's POA
                pl = pl["_finish"]()
            tw = time.perf_counter()
            n = _write_payload(pl, fa, None, counter0, threads)
            timeline.append(("write", tw - t0, time.perf_counter() - t0))
            r2_fut.result()
            del pl
            res.close()
            return n, res

        def write_r2i(res, ix, counter0):
            tw = time.perf_counter()
            _write_payload(_names_payload(res, mine_a[ix]), None, r2, counter0, threads)
            timeline.append(("write_r2i", tw - t0, time.perf_counter() - t0))
        def close_outputs():
            if fa is not None:
                for f in r2_futs + fa_futs:
                    f.exception()
                fa.close()
                r2.close()

        try:
            for k, ix in enumerate(parts):
                res, tcl, (o_a, o_b), tpk = cl[k].result()
                add("t_cluster", tcl)
                add("t_pack", tpk)
                tg = time.perf_counter()
                if dev_orient and getattr(res, "orient_hits", None) is not None:
                    hits, n_hits = res.orient_hits, res.orient_n_hits
                elif dev_orient:
                    hits, n_hits = gpu_orient_segments(res, o_a, o_b, res.sub_off, device=device)
                else:
                    hits, n_hits = orient_fn(o_a, o_b, res.sub_off)
                te = time.perf_counter()
                timeline.append(("orient", tg - t0, te - t0))
                add("t_orient", te - tg)
                asm_fut = host.submit(assemble, res, hits, n_hits)
                poa_futs.append(gpu_poa.submit(poa_job, res, asm_fut, ix))
                if stream_out:
                    r2_futs.append(host.submit(write_r2i, res, ix, n_iso_before))
                    fa_futs.append(writer.submit(write_fasta, poa_futs[-1], n_iso_before, r2_futs[-1]))
                    n_iso_before += res.n_isoforms
            if placed:
                # every chunk is clustered: number this rank's isoforms and place its reads2isoforms.txt
                # blocks (writer thread) while the POA runs
                place_fut = writer.submit(_place_r2i, [names_parts[k] for k in range(len(parts))], comm,
                                          len(roots), out_path, timeline, t0, threads)
        except BaseException:
            close_outputs()
            _close_all(cl, poa_futs)
            raise
        results = []
        if stream_out:
            # one rank: chunks are contiguous runs of the sorted roots and finish in order; both files
            # were written chunk by chunk by the host and writer threads
            written = 0
            try:
                for f in fa_futs:
                    n, res = f.result()
                    results.append(res)
                    written += n
                for f in r2_futs:
                    f.result()
            except BaseException:
                close_outputs()
                _close_all(cl, poa_futs)
                raise
            close_outputs()
            stats["written_isoforms"] = written
        else:
            try:
                for f in poa_futs:
                    pl, res = f.result()
                    results.append(res)
                    payloads.append(pl)
            except BaseException:
                _close_all(cl, poa_futs)
                raise
    if placed:
        tm = time.perf_counter()
        cons = _merge_cons(payloads)
        timeline.append(("merge", tm - t0, time.perf_counter() - t0))
        tw = time.perf_counter()
        stats["written_isoforms"] = _place_fasta(cons, place_fut.result(), comm, len(roots), out_path, threads)
        timeline.append(("write", tw - t0, time.perf_counter() - t0))
        del cons
    elif not stream_out:
        tm = time.perf_counter()
        payload = payloads[0] if len(payloads) == 1 else _merge(payloads)
        if world > 1:
            payload = _gather(payload, comm)
        timeline.append(("merge", tm - t0, time.perf_counter() - t0))
        if rank == 0:
            tw = time.perf_counter()
            with open(out_path + "/Isoform_Consensi.fasta", "wb") as fa, \
                    open(out_path + "/reads2isoforms.txt", "wb") as r2:
                stats["written_isoforms"] = _write_payload(payload, fa, r2, 0, threads)
            timeline.append(("write", tw - t0, time.perf_counter() - t0))
        del payload
    stats["t_total"] = time.perf_counter() - t0
    # host time of the output stages (summed over chunks; streamed writes overlap the POA of later chunks)
    stats["t_write"] = sum(b - a for n, a, b in timeline if n in ("write", "write_r2i"))
    stats["reassembly"] = ("place" if placed else "gather") if world > 1 else "none"
    stats["t_merge"] = sum(b - a for n, a, b in timeline if n == "merge")
    # the chunks' buffers go back to their pools before returning: every kernel that read them has
    # completed (the POA calls are synchronous), and no release can then overlap the next call's kernels
    del payloads
    for r in results:
        r.close()
    stats["t_close"] = time.perf_counter() - t0 - stats["t_total"]
    if hbm:  # what the call's device buffers hold once it is done (caches and POA workspaces, kept for reuse)
        hbm["cache_held_end"] = _lib.cache_trim(device)
        if pctx is not None:
            hbm["poa_ws_held"] = pctx.memory()[1]
    if verbose and rank == 0:
        print("\t" + " ".join(f"{k}={v:.3f}" if isinstance(v, float) else f"{k}={v}" for k, v in stats.items()
                               if not isinstance(v, list)))
    return stats


HBM_PEAK_GBS = 8000.0  # MI355X HBM3E (the POA roofline's peak, as in bench.py)


def metrics(stats: dict, world: int = 1) -> dict:
    """One run's metrics line (written next to Mando.log as JSON): throughput of the whole
    D module and of the POA kernels, with the POA roofline inputs (algorithmic bytes = 1 B per DP cell +
    each read + each consensus, over the launches' HIP-event time)."""
    la = stats.get("poa_launches", [])
    k_ms = sum(x["kernel_ms"] for x in la)
    cells = sum(x["cells"] for x in la)
    alg = sum(x["cells"] + x["read_bytes"] + x["cons_bytes"] for x in la)
    t = stats.get("t_total", 0.0)
    gbs = alg / (k_ms / 1e3) / 1e9 if k_ms > 0 else None
    return {"module": "D", "ranks": world, "loci": stats.get("loci"), "records_rank0": stats.get("records"),
            "isoforms_rank0": stats.get("isoforms"), "poa_groups_rank0": stats.get("poa_groups"),
            "poa_reads_rank0": stats.get("poa_reads"), "wall_s": round(t, 4),
            "records_per_s_rank0": stats["records"] / t if t > 0 and stats.get("records") else None,
            "poa_launches": sum(x["launches"] for x in la), "poa_kernel_ms": round(k_ms, 2), "dp_cells": cells,
            "gcups": cells / (k_ms / 1e3) / 1e9 if k_ms > 0 else None,
            "poa_algorithmic_GBps": gbs, "poa_hbm_roofline_frac": gbs / HBM_PEAK_GBS if gbs else None,
            "phases_s": {k: round(stats[k], 4) for k in ("t_ingest", "t_cluster", "t_orient", "t_assemble", "t_poa")
                         if k in stats}, "chunks": stats.get("chunks")}


def _close_all(cluster_futs, poa_futs) -> None:
    """Error path: wait for every chunk already submitted (clustering, POA) and close the results they
    produced, so no device text or host text buffer outlives the failed call."""
    seen = set()
    for f in list(poa_futs) + list(cluster_futs):
        try:
            r = f.result()
        except BaseException:  # noqa: BLE001 -- the first error is the one re-raised
            continue
        res = r[1] if isinstance(r, tuple) and len(r) == 2 else r[0]
        if id(res) not in seen and hasattr(res, "close"):
            seen.add(id(res))
            res.close()


def _write_payload(payload: dict, fa, r2, counter0: int, threads: int = 0) -> int:
    """Appends a payload's isoforms to both files in output order (sorted roots x IsoDict order,
    defineIsoforms.py:155-166), numbering from counter0 + 1; returns the isoform count.  fa or r2 None:
    that file is skipped (reads2isoforms needs only the clustering, so one rank writes it ahead).  The
    bytes come from mando_format_outputs, one threaded pass straight over the payload arrays."""
    order = np.argsort(payload["iso_root"], kind="stable")
    cons = names = None
    if fa is not None:
        cons = (payload["cons_src"], payload["c_sel"], payload["c_start"], payload["c_len"], payload["c_rc"])
    if r2 is not None:
        names = (payload["name_src"], payload["n_sel"], payload["n_start"], payload["n_len"])
    fasta, r2i = _lib.format_outputs(order, payload["mem_off"], counter0, cons, names, threads=threads)
    if fa is not None:
        _write_big(fa, fasta)
    if r2 is not None:
        _write_big(r2, r2i)
    return int(len(order))


def _write_big(fh, arr: np.ndarray, piece: int = 64 << 20) -> None:
    """Appends arr to the open file: large buffers as parallel pwrite()s of 64 MB pieces (the page-cache
    copy of one write() call runs at ~1.5 GB/s; rank 0 writes a whole 10M-record output at the end of a
    multi-GPU run), small ones with one write()."""
    buf = memoryview(np.ascontiguousarray(arr)).cast("B")
    n = len(buf)
    if n < 4 * piece:
        fh.write(buf)
        return
    from concurrent.futures import ThreadPoolExecutor

    fh.flush()
    fd, at = fh.fileno(), fh.tell()

    def one(o):
        v = buf[o:o + piece]
        done = 0
        while done < len(v):
            done += os.pwrite(fd, v[done:], at + o + done)

    with ThreadPoolExecutor(max_workers=8) as ex:
        list(ex.map(one, range(0, n, piece)))
    fh.seek(at + n)


def _poa_chunk(res: cluster.ClusterResult, root_idx: Sequence[int], prep, run_poa, stats: dict, lock,
               launches: list | None = None):
    """POA of one oriented chunk; returns its writer payload, or {"_finish": f} when a part still runs on
    the wide context (f() waits for it and returns the payload)."""
    asm, p_grp = prep[0], prep[-1]
    t3 = time.perf_counter()
    parts = run_poa(res, prep)
    t4 = time.perf_counter()
    with lock:
        stats["poa_groups"] += int(len(asm.poa_iso))
        stats["records"] += int(res.n_records)
        stats["poa_reads"] += int(p_grp[-1])
        stats["t_poa"] += t4 - t3
    base = _names_payload(res, root_idx)

    def finish():
        # consensus of every isoform as a byte segment: POA output, else (<=2 sequences, or an empty POA
        # result) the first emission, re-bound (SDC:911-926)
        n_iso = res.n_isoforms
        fe = asm.first_emit
        c_sel = np.zeros(n_iso, dtype=np.int16)                     # 0: read text, k: POA part k
        c_start = res.seq_off[asm.e_rec[fe]] if n_iso else np.zeros(0, np.int64)
        c_len = res.seq_len[asm.e_rec[fe]].astype(np.int64) if n_iso else np.zeros(0, np.int64)
        c_rc = (asm.e_sign[fe] == -1).astype(np.int8) if n_iso else np.zeros(0, np.int8)
        src, infos = [res.text], []
        for part in parts:
            got = part.result() if isinstance(part, _Pending) else part
            cons, cons_off, gidx = got[:3]
            if len(got) > 3 and got[3] is not None:
                infos.append(got[3])
            plen = np.diff(cons_off)
            use = plen > 0
            g = np.flatnonzero(use) if gidx is None else gidx[use]
            pi = asm.poa_iso[g]
            c_sel[pi] = len(src)
            c_start[pi] = cons_off[:-1][use]
            c_len[pi] = plen[use]
            c_rc[pi] = 0
            src.append(cons)
        if infos and launches is not None:
            # the split chunk's parts as one entry: their launches started together, so the pair's time
            # is the longer one's (as for the kinds of one batch)
            with lock:
                launches.append({"cells": sum(x.get("cells", 0) for x in infos),
                                 "kernel_ms": max(x["kernel_ms"] for x in infos),
                                 "launches": sum(x.get("launches", 0) for x in infos),
                                 "read_bytes": sum(x["read_bytes"] for x in infos),
                                 "cons_bytes": sum(x["cons_bytes"] for x in infos),
                                 "reads": sum(x["reads"] for x in infos)})
        with lock:
            stats["isoforms"] += n_iso
        return dict(base, cons_src=src, c_sel=c_sel, c_start=c_start, c_len=c_len, c_rc=c_rc)

    if any(isinstance(p, _Pending) for p in parts):
        return {"_finish": finish}
    return finish()


def _names_payload(res: cluster.ClusterResult, root_idx: Sequence[int]) -> dict:
    """The part of a chunk's writer payload that the clustering alone fixes (isoform order, member names)."""
    ri = np.asarray(root_idx, dtype=np.int64)
    n_mem = int(res.mem_off[-1])
    return dict(iso_root=ri[res.iso_locus] if res.n_isoforms else np.zeros(0, np.int64), name_src=[res.text],
                n_sel=np.zeros(n_mem, np.int16), n_start=res.name_off[res.mem],
                n_len=res.name_len[res.mem].astype(np.int64), mem_off=res.mem_off)


def _compact(payload: dict) -> dict:
    """One consensus buffer and one name buffer (the referenced bytes gathered out of every source), so a
    rank ships only its results."""
    ct, co = _lib.pack_segments(payload["cons_src"], payload["c_start"], payload["c_len"], sel=payload["c_sel"],
                                rc=payload["c_rc"])
    names, noff = _lib.pack_segments(payload["name_src"], payload["n_start"], payload["n_len"], sel=payload["n_sel"])
    n_iso, n_mem = len(payload["c_len"]), len(payload["n_len"])
    return dict(iso_root=payload["iso_root"], cons_src=[ct], c_sel=np.zeros(n_iso, np.int16), c_start=co[:-1],
                c_len=payload["c_len"], c_rc=np.zeros(n_iso, np.int8), name_src=[names],
                n_sel=np.zeros(n_mem, np.int16), n_start=noff[:-1], n_len=payload["n_len"], mem_off=payload["mem_off"])


def _compact_names(p: dict) -> dict:
    """A names payload with its member names copied into one buffer (independent of the chunk's text)."""
    names, noff = _lib.pack_segments(p["name_src"], p["n_start"], p["n_len"], sel=p["n_sel"])
    return dict(iso_root=np.array(p["iso_root"], copy=True), mem_off=np.array(p["mem_off"], copy=True),
                name_src=[names], n_sel=np.zeros(len(p["n_len"]), np.int16), n_start=noff[:-1],
                n_len=np.array(p["n_len"], copy=True))


def _compact_cons(p: dict) -> dict:
    """The consensus part of a payload, copied into one buffer (the names were copied at clustering)."""
    ct, co = _lib.pack_segments(p["cons_src"], p["c_start"], p["c_len"], sel=p["c_sel"], rc=p["c_rc"])
    n_iso = len(p["c_len"])
    return dict(iso_root=p["iso_root"], cons_src=[ct], c_sel=np.zeros(n_iso, np.int16), c_start=co[:-1],
                c_len=np.array(p["c_len"], copy=True), c_rc=np.zeros(n_iso, np.int8))


def _merge_cons(parts: list) -> tuple:
    """The chunks' consensi (compacted, chunk order) as one (srcs, sel, start, len, rc) tuple."""
    sel = [np.full(len(p["c_len"]), k, np.int16) for k, p in enumerate(parts)]
    cat = lambda f, dt: np.concatenate([p[f] for p in parts]).astype(dt) if parts else np.zeros(0, dt)
    return ([p["cons_src"][0] for p in parts], np.concatenate(sel) if sel else np.zeros(0, np.int16),
            cat("c_start", np.int64), cat("c_len", np.int64), np.zeros(sum(len(s) for s in sel), np.int8))


def _exchange_per_root(comm, n_roots: int, roots: np.ndarray, *vals: np.ndarray) -> list:
    """One all-gather of (root, values...) for this rank's roots; returns each value as a dense per-root
    array over all ranks (every root belongs to one rank)."""
    m = len(roots)
    blob = np.concatenate([np.array([m], np.int64), np.asarray(roots, np.int64)]
                          + [np.asarray(v, np.int64) for v in vals]).view(np.uint8)
    allb, counts = comm.allgather_bytes(blob)
    out = [np.zeros(n_roots, np.int64) for _ in vals]
    base = 0
    for c in counts:
        part = allb[base:base + int(c)].view(np.int64)
        base += int(c)
        k = int(part[0])
        r = part[1:1 + k]
        for j, o in enumerate(out):
            o[r] = part[1 + k * (j + 1):1 + k * (j + 2)]
    return out


def _alltoallv(comm, parts: list) -> list:
    """comm.alltoallv, or (in-process stand-ins with only allgather_bytes) one all-gather of every rank's
    parts with per-rank headers, of which each rank keeps the parts addressed to it."""
    if hasattr(comm, "alltoallv"):
        return comm.alltoallv(parts)
    world, me = comm.world, comm.rank
    parts = [np.ascontiguousarray(p, dtype=np.uint8).ravel() for p in parts]
    hdr = np.array([p.size for p in parts], dtype=np.int64)
    allb, cnt = comm.allgather_bytes(np.concatenate([hdr.view(np.uint8)] + parts))
    out, base = [], 0
    for r in range(world):
        blob = allb[base:base + int(cnt[r])]
        base += int(cnt[r])
        if blob.size < 8 * world:  # (a stand-in rank that has not contributed yet)
            out.append(np.zeros(0, np.uint8))
            continue
        h = blob[:8 * world].view(np.int64)
        a = 8 * world + int(h[:me].sum())
        out.append(blob[a:a + int(h[me])])
    return out


def _range_bounds(total: int, world: int) -> np.ndarray:
    """Rank r writes bytes [b[r], b[r+1]) of an output file: equal shares, cut at 4 KiB pages."""
    b = np.array([(total * r // world) & ~4095 for r in range(world)] + [total], dtype=np.int64)
    b[0] = 0
    return np.maximum.accumulate(b)


def _place(path: str, buf: np.ndarray, src: np.ndarray, roots: np.ndarray, sizes: np.ndarray,
           g_sizes: np.ndarray, comm, threads: int = 0) -> None:
    """Range placement of one output file: this rank's per-root blocks of buf (source offsets src, roots
    `roots`, sizes `sizes`; g_sizes = every root's block size over all ranks) go to the ranks that own
    their bytes of the file -- rank r owns one contiguous range (_range_bounds) -- in one personalised
    exchange, and each rank writes its range in one piece.  Ranks writing interleaved small blocks into
    one file contend for its pages: 8 processes placing config 4's 1 GB FASTA that way took 0.74 s on the
    GPU box against 0.12 s for one contiguous range each.  The file's size is the total of
    every rank's blocks (each rank sets it), so no rank truncates another's bytes."""
    world, me = comm.world, comm.rank
    goff = np.zeros(len(g_sizes) + 1, np.int64)
    np.cumsum(g_sizes, out=goff[1:])
    total = int(goff[-1])
    bnd = _range_bounds(total, world)
    # this rank's blocks cut into pieces at the range bounds, by destination rank
    dst = goff[np.asarray(roots, dtype=np.int64)]
    src = np.asarray(src, dtype=np.int64)
    ln = np.asarray(sizes, dtype=np.int64)
    keep = ln > 0
    dst, src, ln = dst[keep], src[keep], ln[keep]
    r0 = np.searchsorted(bnd, dst, side="right") - 1
    r1 = np.searchsorted(bnd, dst + ln - 1, side="right") - 1
    cross = np.flatnonzero(r1 > r0)
    if len(cross):  # blocks across a bound (at most world - 1 of them): one piece per range
        pd, ps, pl = [], [], []
        for i in cross:
            a, b, s0 = int(dst[i]), int(dst[i] + ln[i]), int(src[i])
            for r in range(int(r0[i]), int(r1[i]) + 1):
                lo, hi = max(a, int(bnd[r])), min(b, int(bnd[r + 1]))
                if hi > lo:
                    pd.append(lo)
                    ps.append(s0 + lo - a)
                    pl.append(hi - lo)
        whole = np.ones(len(dst), dtype=bool)
        whole[cross] = False
        dst, src, ln = (np.concatenate([v[whole], np.array(x, dtype=np.int64)])
                        for v, x in ((dst, pd), (src, ps), (ln, pl)))
    rk = np.searchsorted(bnd, dst, side="right") - 1
    order = np.argsort(dst, kind="stable")  # file order, so by destination rank too
    dst, src, ln, rk = dst[order], src[order], ln[order], rk[order]
    cut = np.searchsorted(rk, np.arange(world + 1))
    payload, _ = _lib.pack_segments([buf], src, ln, threads=threads)
    boff = np.concatenate([[0], np.cumsum(ln)])
    meta = [np.stack([dst[cut[r]:cut[r + 1]], ln[cut[r]:cut[r + 1]]], axis=1).astype(np.int64).view(np.uint8)
            for r in range(world)]
    data = [payload[boff[cut[r]]:boff[cut[r + 1]]] for r in range(world)]
    got_meta = _alltoallv(comm, meta)
    got_data = _alltoallv(comm, data)
    lo, hi = int(bnd[me]), int(bnd[me + 1])
    rb = np.zeros(max(hi - lo, 1), dtype=np.uint8)
    # in-process stand-in communicators (tests without alltoallv, tools/rank_rehearsal.py's `standin`
    # transport) deliver incomplete data in their early passes, whose pieces are dropped; over a real
    # transport every piece must land inside this rank's range and the pieces must tile it, or the
    # exchange disagreed and the file would carry zero bytes
    standin = getattr(comm, "standin", False) or not hasattr(comm, "alltoallv")
    sel, starts, lens, outs = [], [], [], []
    got = 0
    for r in range(world):
        m = np.ascontiguousarray(got_meta[r]).view(np.int64).reshape(-1, 2)
        if not len(m):
            continue
        st = np.concatenate([[0], np.cumsum(m[:, 1])[:-1]])
        ok = (m[:, 0] >= lo) & (m[:, 0] + m[:, 1] <= hi) & (st + m[:, 1] <= got_data[r].size)
        if not standin and not ok.all():
            raise RuntimeError(f"range placement of {os.path.basename(path)}: rank {r} sent {int((~ok).sum())} "
                               f"piece(s) outside rank {me}'s range [{lo}, {hi}) or beyond its data")
        got += int(m[ok, 1].sum())
        sel.append(np.full(int(ok.sum()), r, np.int8))
        starts.append(st[ok])
        lens.append(m[ok, 1])
        outs.append(m[ok, 0] - lo)
    if not standin and got != hi - lo:
        raise RuntimeError(f"range placement of {os.path.basename(path)}: rank {me} received {got} bytes for its "
                           f"range [{lo}, {hi}) of {hi - lo}")
    if sel:
        _lib.pack_segments([np.ascontiguousarray(g) if g.size else np.zeros(1, np.uint8) for g in got_data],
                           np.concatenate(starts), np.concatenate(lens), sel=np.concatenate(sel), threads=threads,
                           out=rb, out_off=np.concatenate(outs))
    fd = os.open(path, os.O_RDWR | os.O_CREAT, 0o644)  # read-write: mando_write_blocks maps the file
    try:
        os.ftruncate(fd, total)
        if hi > lo:
            _lib.write_blocks(fd, rb, np.zeros(1, np.int64), np.array([lo], np.int64), np.array([hi - lo], np.int64),
                              threads=threads)
    finally:
        os.close(fd)


def _place_r2i(parts: list, comm, n_roots: int, out_path: str, timeline: list, t0: float,
               threads: int = 0) -> tuple:
    """Placement reassembly, clustering half (defineIsoforms.py:155-166 numbers isoforms in sorted-root
    order across all loci): the ranks exchange per-root isoform counts, number their own isoforms from
    them and place their reads2isoforms.txt blocks.  Returns what the FASTA half needs."""
    tw = time.perf_counter()
    cat = lambda f: np.concatenate([p[f] for p in parts]) if parts else np.zeros(0, np.int64)
    iso_root = cat("iso_root")
    mem_off = np.zeros(1, np.int64)
    if parts:
        mem_off = np.concatenate([np.zeros(1, np.int64)] + [p["mem_off"][1:] + b for p, b in zip(
            parts, np.cumsum([0] + [int(p["mem_off"][-1]) for p in parts[:-1]]))])
    names = ([p["name_src"][0] for p in parts],
             np.concatenate([np.full(len(p["n_len"]), k, np.int16) for k, p in enumerate(parts)])
             if parts else np.zeros(0, np.int16), cat("n_start"), cat("n_len"))
    order = np.argsort(iso_root, kind="stable")
    rs = iso_root[order]
    ur, first, cnt = np.unique(rs, return_index=True, return_counts=True)
    g_cnt, = _exchange_per_root(comm, n_roots, ur, cnt)
    kbase = np.zeros(n_roots + 1, np.int64)
    np.cumsum(g_cnt, out=kbase[1:])
    k = kbase[rs] + 1 + (np.arange(len(rs), dtype=np.int64) - np.repeat(first, cnt))
    _, r2i, _, ro = _lib.format_outputs(order, mem_off, 0, None, names, threads=threads, iso_k=k, offsets=True)
    sz = ro[first + cnt] - ro[first]
    g_sz, = _exchange_per_root(comm, n_roots, ur, sz)
    _place(out_path + "/reads2isoforms.txt", r2i, ro[first], ur, sz, g_sz, comm, threads)
    timeline.append(("write_r2i", tw - t0, time.perf_counter() - t0))
    return order, mem_off, k, ur, first, cnt


def _place_fasta(cons: tuple, numbered: tuple, comm, n_roots: int, out_path: str, threads: int = 0) -> int:
    """Placement reassembly, POA half: per-root FASTA sizes exchanged, blocks placed, then one barrier
    (every rank's blocks of both files are written when any rank returns)."""
    order, mem_off, k, ur, first, cnt = numbered
    fasta, _, fo, _ = _lib.format_outputs(order, mem_off, 0, cons, None, threads=threads, iso_k=k, offsets=True)
    sz = fo[first + cnt] - fo[first]
    g_sz, = _exchange_per_root(comm, n_roots, ur, sz)
    _place(out_path + "/Isoform_Consensi.fasta", fasta, fo[first], ur, sz, g_sz, comm, threads)
    comm.barrier()
    return int(len(order))


_FIELDS = ("iso_root", "c_start", "c_len", "n_start", "n_len", "mem_off")


def _gather(payload: dict, comm) -> dict:
    """Reassembly on rank 0: one gather of each rank's compacted results to the writer
    (RCCL point-to-point sends over xGMI between GPUs, the rendezvous sockets on CPU).  Each rank ships its
    isoforms' root indices, consensus bytes and member names; only rank 0 receives and unpacks them."""
    p = _compact(payload)
    arrays = [np.ascontiguousarray(p[f]) for f in _FIELDS] + [p["cons_src"][0], p["name_src"][0]]
    hdr = np.array([a.nbytes for a in arrays] + [a.dtype.num for a in arrays], dtype=np.int64)
    blob = np.concatenate([hdr.view(np.uint8)] + [a.view(np.uint8).ravel() for a in arrays])
    allb, counts = comm.gather_bytes(blob)
    if comm.rank != 0:
        return payload
    parts = []
    na = len(arrays)
    base = 0
    for k in range(comm.world):
        raw = allb[base:base + int(counts[k])]
        base += int(counts[k])
        h = raw[: 16 * na].view(np.int64)
        sizes, kinds = h[:na], h[na:]
        pos = 16 * na
        arrs = []
        for sz, kd in zip(sizes, kinds):
            arrs.append(raw[pos:pos + sz].view(_dtype_of(int(kd))))
            pos += int(sz)
        d = dict(zip(_FIELDS, arrs[:len(_FIELDS)]))
        n_iso, n_mem = len(d["c_len"]), len(d["n_len"])
        d.update(cons_src=[arrs[len(_FIELDS)]], c_sel=np.zeros(n_iso, np.int16), c_rc=np.zeros(n_iso, np.int8),
                 name_src=[arrs[len(_FIELDS) + 1]], n_sel=np.zeros(n_mem, np.int16))
        parts.append(d)
    return _merge(parts)


def _merge(payloads: list) -> dict:
    """Concatenate payloads: index arrays appended, byte sources listed (selectors rebased), offsets of
    members rebased; no bytes are copied."""
    if len(payloads) == 1:
        return payloads[0]
    out = {f: [] for f in ("iso_root", "c_sel", "c_start", "c_len", "c_rc", "n_sel", "n_start", "n_len", "mem_off")}
    cons_src, name_src = [], []
    bm = 0
    for d in payloads:
        out["iso_root"].append(d["iso_root"])
        out["c_sel"].append(d["c_sel"].astype(np.int16) + len(cons_src))
        out["c_start"].append(d["c_start"])
        out["c_len"].append(d["c_len"])
        out["c_rc"].append(d["c_rc"])
        out["n_sel"].append(d["n_sel"].astype(np.int16) + len(name_src))
        out["n_start"].append(d["n_start"])
        out["n_len"].append(d["n_len"])
        out["mem_off"].append(d["mem_off"][1:] + bm if len(out["mem_off"]) else d["mem_off"] + bm)
        bm += int(d["mem_off"][-1])
        cons_src += list(d["cons_src"])
        name_src += list(d["name_src"])
    merged = {f: np.concatenate(v) for f, v in out.items()}
    merged["cons_src"] = cons_src
    merged["name_src"] = name_src
    return merged


def _dtype_of(num: int):
    for t in (np.int64, np.int32, np.int8, np.uint8):
        if np.dtype(t).num == num:
            return np.dtype(t)
    raise ValueError(num)


def parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(description="MI355X-native defineIsoforms (Mandalorion D module)")
    ap.add_argument("--infile", "-i", type=str)
    ap.add_argument("--path", "-p", type=str)
    ap.add_argument("--cutoff", "-c", type=float)
    ap.add_argument("--genome_file", "-g", type=str)
    ap.add_argument("--splice_site_width", "-w", type=int)
    ap.add_argument("--minimum_read_count", "-m", type=int)
    ap.add_argument("--white_list_polyA", "-W", type=str)
    ap.add_argument("--numThreads", "-n", type=str)
    ap.add_argument("--junctions", "-j", type=str)
    ap.add_argument("--upstream_buffer", "-u", type=str)
    ap.add_argument("--downstream_buffer", "-d", type=str)
    ap.add_argument("--abpoa", "-a", type=str, help="accepted for CLI compatibility; consensus runs on the GPU")
    ap.add_argument("--seed", type=int, default=int(os.environ.get("MANDO_RNG_SEED", "0")),
                    help="numpy global RNG state every locus starts from (the reference leaves it unseeded)")
    ap.add_argument("--device", type=int, default=int(os.environ.get("LOCAL_RANK", "0")))
    return ap


def main(argv: list[str] | None = None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    ap = parser()
    if not argv:
        ap.print_help()
        return 0
    a = ap.parse_args(argv)
    comm = None
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        from .comm import Comm

        comm = Comm.from_env(device=a.device)
    try:
        define_isoforms(a.path, cutoff=float(a.cutoff), genome_file=a.genome_file,
                        splice_site_width=int(a.splice_site_width), minimum_read_count=int(a.minimum_read_count),
                        white_list_polyA=a.white_list_polyA.split(","), threads=int(a.numThreads),
                        junctions=a.junctions, upstream_buffer=int(a.upstream_buffer),
                        downstream_buffer=int(a.downstream_buffer), seed=a.seed, device=a.device, comm=comm,
                        verbose=True)
    finally:
        if comm is not None:
            comm.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
