#!/usr/bin/env python3
"""Benchmark of the D module (`Mando.py -M D`, i.e. defineIsoforms.py) on MI355X — SURVEY.md §8(d).

Headline (`value`): PSL records / wall second of the whole D module — locus PSL files on disk ->
clustering -> orientation (HIP) -> batched POA consensus (HIP) -> Isoform_Consensi.fasta +
reads2isoforms.txt closed — by default on BASELINE.json configs[3], the north star's 10M-read strong-scaling
set, which fits one MI355X: 200,000 synthetic loci x 40-60 reads of 2-4 kb (80 % R2C2 / 20 % PacBio error
profiles, half of the reads on the '-' strand; ~10M PSL records, 62 GB of locus text), seed 20250117.
`--workload config3` is configs[2] (20,000 loci x 50 R2C2 reads of ~3 kb, 1M records).  One step = one
full `define_isoforms` pass over the data set; the clock runs from the start of locus ingest until both
output files are closed.

Multi-GPU (`--gpus N`, one process per GPU under the driver's launcher): strong scaling.  The same data
set is sharded over the ranks by the §8(e) cost estimate (LPT); each rank clusters, orients and runs
the POA on its loci; the ranks exchange per-root isoform counts and byte sizes (RCCL all-gathers over
xGMI, libmando mando_comm_*) and each writes its own roots' bytes into the shared output files.
value = records / max-over-ranks wall time.

Also reported: the POA kernel's roofline (algorithmic bytes per launch / launch time from HIP events on
the launch stream), the POA kernel rate (reads through POA / kernel time), and `cpu_baseline`: the same
driver with the CPU restatements (oracle/) injected for orientation and POA, on a bounded sample of
the same loci, on the box's host cores (rank 0, N=1 only).  That sample's GPU output must be
byte-identical to the CPU run's.

Launch: under a launcher (WORLD_SIZE set) each process is one rank.  `--gpus N` without one spawns the N
rank processes itself (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set per child, before anything in the
parent touches a GPU) and exits with the worst child status.  With N > 1 every rank must end up on RCCL
(`comm.backend == "rccl"`), else the run fails; `n_gpus` is the communicator's world size.
`--check-launch` stops after the rendezvous, the data and the LPT plan (no GPU compute): it prints the
ranks, their backend and their loci, and runs without a device (host transport).

Output parity: after the timed steps the two files of the last step are hashed and compared with
tests/golden/fullsize_hashes.json (the oracle's output on the same full-size workload, computed in the
build container by tests/golden/make_fullsize_hashes.py); a mismatch fails the run.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import resource
import shutil
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X, /opt/skills/guides/MI355X_MICROARCH.md "Chip-level parameters"
FULLSIZE_HASHES = os.path.join(ROOT, "tests", "golden", "fullsize_hashes.json")
# the sources whose code the PMC traffic of profiles/pmc_latest.json describes
POA_SOURCES = ("poa_kernel.hip", "poa_kernel.h", "seed_kernel.hip", "capi.hip")


def poa_sources_sha() -> str:
    h = hashlib.sha256()
    for f in POA_SOURCES:
        with open(os.path.join(ROOT, "mandalorion_amd", "csrc", f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


def plan_signature() -> dict:
    """The D driver's chunk-plan constants: a PMC file measured under another plan describes other launches."""
    from mandalorion_amd import define

    return {"chunk_bytes": define._CHUNK_BYTES, "big_chunk_bytes": define._BIG_CHUNK_BYTES,
            "big_input_bytes": define._BIG_INPUT_BYTES, "two_chunk_bytes": define._TWO_CHUNK_BYTES,
            "min_loci_chunked": define._MIN_LOCI_CHUNKED}


def host_cores() -> dict:
    """The host CPUs this process may use: affinity, capped by the cgroup CPU quota (cpu.max), and the
    machine's count (os.cpu_count(), which on the GPU box is the whole host, many times our share)."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) // int(per)))
    except (OSError, ValueError):
        pass
    usable = min(aff, quota) if quota else aff
    return {"nproc": os.cpu_count(), "affinity": aff, "cgroup_quota": quota, "usable": usable}

WORKLOADS = {
    # BASELINE.json configs[1]: SIRV-like spike-in set, 7 genes x ~10 isoforms, ~50k R2C2 reads
    "config2": dict(loci=7, reads=(6500, 7500), exons=(10, 14), exon_len=(60, 200), isoforms=(9, 11), pacbio_frac=0.0,
                    rev_frac=0.3,
                    text="config2: SIRV-like, 7 loci x ~7,000 synthetic R2C2 reads (10-14 exons of 60-200 nt, 9-11 "
                         "isoforms/locus, 30% '-' strand), ~50k PSL records, Mando.py -M D"),
    # BASELINE.json configs[2]: 1M synthetic ~3 kb R2C2 reads over 20k loci
    "config3": dict(loci=20000, reads=(50, 50), exon_len=(200, 500), pacbio_frac=0.0, rev_frac=0.3,
                    text="config3: 20,000 loci x 50 synthetic R2C2 reads (~3 kb, 5-12 exons of 200-500 nt, "
                         "1-3 isoforms/locus, 30% '-' strand), 1M PSL records, Mando.py -M D"),
    # BASELINE.json configs[4]: stress, 200-read-deep loci at ~8 kb (POA sees 100 per isoform, abPOA -S)
    "config5": dict(loci=100, reads=(200, 200), exons=(8, 10), exon_len=(850, 1000), isoforms=(1, 1), pacbio_frac=0.0,
                    rev_frac=0.3,
                    text="config5: 100 loci x 200 synthetic R2C2 reads of ~8.5 kb (1 isoform/locus, subsampled to "
                         "100, median >= 8000 nt -> -S), 20k PSL records, Mando.py -M D"),
    # BASELINE.json configs[3]: 10M mixed R2C2 + PacBio 2-4 kb reads (~200k gencode-like loci)
    "config4": dict(loci=200000, reads=(40, 60), exon_len=(130, 570), pacbio_frac=0.2, rev_frac=0.5,
                    text="config4: 200,000 loci x 40-60 synthetic reads (2-4 kb, 80% R2C2 / 20% PacBio error "
                         "rates, 50% '-' strand), ~10M PSL records, Mando.py -M D"),
}


def log(msg: str) -> None:
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


class heartbeat:
    """A line on stderr every 30 s while a long, silent call (data generation) runs."""

    def __init__(self, what: str):
        self.what = what

    def __enter__(self):
        import threading

        self.stop = threading.Event()
        t0 = time.perf_counter()

        def beat():
            while not self.stop.wait(30.0):
                log(f"{self.what}: {time.perf_counter() - t0:.0f} s")

        self.th = threading.Thread(target=beat, daemon=True)
        self.th.start()
        return self

    def __exit__(self, *exc):
        self.stop.set()
        self.th.join()
        return False


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="config4")
    ap.add_argument("--loci", type=int, default=0, help="override the workload's locus count")
    ap.add_argument("--data-dir", default="", help="where the synthetic tmp_SS goes (default $TMPDIR)")
    ap.add_argument("--threads", type=int, default=0, help="host threads per rank (0: 16 / ranks per node)")
    ap.add_argument("--cpu-loci", type=int, default=2000, help="cpu_baseline sample size (loci): 10-30 s of CPU work")
    ap.add_argument("--cpu-threads", type=int, default=0, help="cpu_baseline threads (0: the usable host cores)")
    ap.add_argument("--check-launch", action="store_true",
                    help="launch, rendezvous, data and shard plan only (no GPU compute); prints the ranks")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--share", type=int, default=0,
                    help="one GPU runs rank 0's loci of an N-rank LPT plan (the per-rank load of an N-GPU run)")
    ap.add_argument("--pmc-json", default=os.path.join(ROOT, "profiles", "pmc_latest.json"))
    return ap.parse_args()


def gen_data(d: str, wl: dict, n_loci: int, threads: int) -> int:
    """Synthetic tmp_SS (libmando_synth); a marker file caches the record count across runs."""
    from mandalorion_amd import synth

    marker = os.path.join(d, "records.txt")
    if os.path.exists(marker):
        return int(open(marker).read())
    shutil.rmtree(os.path.join(d, "tmp_SS"), ignore_errors=True)
    extra = {k: wl[k] for k in ("exons", "isoforms") if k in wl}
    n = synth.write_loci(os.path.join(d, "tmp_SS"), n_loci, reads=wl["reads"], exon_len=wl["exon_len"],
                         threads=threads, pacbio_frac=wl["pacbio_frac"], rev_frac=wl["rev_frac"], **extra)
    with open(marker + ".tmp", "w") as fh:
        fh.write(str(n))
    os.replace(marker + ".tmp", marker)
    return n


def cpu_fns(threads: int, simd: bool = True, poa_stats: dict | None = None):
    """orient_fn / consensus_fn over the CPU restatements (oracle/), groups split over host threads
    (ctypes drops the GIL inside the C calls).  simd: the POA restatement's AVX2 int16 build
    (oracle/poa_simd.c, byte-identical to poa_ref.c); poa_stats (optional) accumulates the POA calls'
    wall seconds and DP cells."""
    from concurrent.futures import ThreadPoolExecutor

    from oracle import orient as oref
    from oracle import poa as opoa

    pool = ThreadPoolExecutor(max_workers=threads)

    def split(seq_off, grp_off, k):
        lens = np.diff(seq_off)
        cost = np.add.reduceat(lens, grp_off[:-1]).astype(np.float64) if len(lens) else np.zeros(0)
        cost *= np.maximum(1, np.diff(grp_off))
        cs = np.cumsum(cost)
        cuts = [0] + [int(np.searchsorted(cs, cs[-1] * i / k)) for i in range(1, k)] + [len(grp_off) - 1]
        cuts = sorted(set(min(max(c, 0), len(grp_off) - 1) for c in cuts))
        return [(cuts[i], cuts[i + 1]) for i in range(len(cuts) - 1) if cuts[i + 1] > cuts[i]]

    def sub(seqs, seq_off, grp_off, a, b):
        r0, r1 = grp_off[a], grp_off[b]
        return seqs, seq_off[r0:r1 + 1], grp_off[a:b + 1] - r0

    def orient_fn(seqs, seq_off, grp_off):
        parts = split(seq_off, grp_off, 4 * threads)
        res = list(pool.map(lambda ab: oref.orient_packed(*sub(seqs, seq_off, grp_off, *ab)), parts))
        if not res:
            return oref.orient_packed(seqs, seq_off, grp_off)
        return np.concatenate([r[0] for r in res]), np.concatenate([r[1] for r in res])

    def consensus_fn(seqs, seq_off, grp_off, seeding):
        t0 = time.perf_counter()
        cells = np.zeros(max(1, len(grp_off) - 1), dtype=np.int64)
        parts = split(seq_off, grp_off, 4 * threads)
        if not parts:
            return opoa.consensus_packed(seqs, seq_off, grp_off, simd=simd)

        def one(ab):
            c = np.zeros(max(1, ab[1] - ab[0]), dtype=np.int64)
            r = opoa.consensus_packed(*sub(seqs, seq_off, grp_off, *ab), simd=simd, cells_out=c,
                                      seeding=None if seeding is None else seeding[ab[0]:ab[1]])
            cells[ab[0]:ab[1]] = c[:ab[1] - ab[0]]
            return r

        res = list(pool.map(one, parts))
        if poa_stats is not None:
            poa_stats["s"] = poa_stats.get("s", 0.0) + time.perf_counter() - t0
            poa_stats["cells"] = poa_stats.get("cells", 0) + int(cells[:len(grp_off) - 1].sum())
        cons = np.concatenate([c[:int(o[-1])] for c, o in res])
        off = [np.zeros(1, dtype=np.int64)]
        base = 0
        for _, o in res:
            off.append(o[1:] + base)
            base += int(o[-1])
        return cons, np.concatenate(off)

    return orient_fn, consensus_fn, pool


SHARE = None  # (rank, N) with --share N: every D pass runs that rank's loci only


def run_define(d, threads, device, comm=None, **kw):
    from mandalorion_amd import define

    if SHARE is not None and comm is None and "share" not in kw and "orient_fn" not in kw:
        kw["share"] = SHARE
    return define.define_isoforms(d, threads=threads, device=device, comm=comm, **kw)


def sample_dir(src: str, dst: str, n: int) -> int:
    """dst/tmp_SS = symlinks to the first n locus files of src (sorted roots), for the CPU baseline."""
    from mandalorion_amd import define

    roots = define._roots(os.path.join(src, "tmp_SS"))[:n]
    shutil.rmtree(dst, ignore_errors=True)
    os.makedirs(os.path.join(dst, "tmp_SS"))
    recs = 0
    for r in roots:
        f = os.path.join(src, "tmp_SS", r + ".psl")
        os.symlink(f, os.path.join(dst, "tmp_SS", r + ".psl"))
        with open(f, "rb") as fh:
            recs += sum(1 for _ in fh)
    return recs


def sha(path):
    return hashlib.sha256(open(path, "rb").read()).hexdigest()


def cpu_baseline(data: str, n_loci: int, threads: int):
    """The restated CPU baseline (SURVEY.md §8(d) option 2): host clustering + oracle/ orientation and
    POA on `threads` host threads, on the first n_loci loci of the same data set."""
    d = os.path.join(data, "cpu_sample")
    recs = sample_dir(data, d, n_loci)
    ps: dict = {}
    of, cf, pool = cpu_fns(threads, simd=True, poa_stats=ps)
    try:
        t0 = time.perf_counter()
        from oracle import cluster as ocl

        st = run_define(d, threads, 0, orient_fn=of, consensus_fn=cf, cluster_fn=ocl.cluster_loci)
        wall = time.perf_counter() - t0
    finally:
        pool.shutdown()
    gcups = ps.get("cells", 0) / ps["s"] / 1e9 if ps.get("s") else None
    out = {"value": recs / wall, "unit": "records/s", "cores": threads, "kind": "simd-port",
           "sample": f"first {n_loci} loci ({recs} PSL records, {st['poa_reads']} POA reads) of this workload through "
                     f"the same D driver with oracle/orient_ref.c (C restatement of mappy map-ont), "
                     f"oracle/poa_simd.c (the abPOA v1.4.1 restatement with its DP rows in AVX2 int16 lanes, as "
                     f"abPOA vectorises them; byte-identical to oracle/poa_ref.c) and oracle/cluster_ref.cpp "
                     f"(clustering) on {threads} host threads; {wall:.1f} s wall",
           # the POA stage alone: its wall seconds on the host threads and its DP cells per second
           "poa_s": round(ps.get("s", 0.0), 3), "poa_gcups": gcups,
           "poa_gcups_per_core": gcups / threads if gcups else None}
    hashes = (sha(os.path.join(d, "Isoform_Consensi.fasta")), sha(os.path.join(d, "reads2isoforms.txt")))
    return out, d, hashes


def spawn_ranks(n: int) -> int:
    """`--gpus N` without a launcher: N rank processes of this script, one per GPU (LOCAL_RANK = GPU),
    started before this parent touches a GPU; returns the worst exit status."""
    import socket
    import subprocess

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    codes = [p.wait() for p in procs]
    return max(codes, key=abs) if any(codes) else 0


def page_cache_resident(files: list, stride: int = 1) -> dict:
    """Share of the locus files' pages resident in the page cache (mincore over a read-only mapping of
    every stride-th file; the mapping faults nothing in), plus the cgroup's file-cache bytes: the timed
    steps read the locus text from the page cache, so a box with less free RAM would read from disk."""
    import ctypes
    import mmap

    libc = ctypes.CDLL(None, use_errno=True)
    libc.mmap.restype = ctypes.c_void_p
    libc.mmap.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_long]
    libc.munmap.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    libc.mincore.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
    pg = os.sysconf("SC_PAGE_SIZE")
    fail = ctypes.c_void_p(-1).value
    tot = res = nf = 0
    for f in files[::max(1, stride)]:
        fd = os.open(f, os.O_RDONLY)
        try:
            n = os.fstat(fd).st_size
            if n == 0:
                continue
            a = libc.mmap(None, n, mmap.PROT_READ, mmap.MAP_SHARED, fd, 0)
            if a is None or a == fail:
                continue
            npg = (n + pg - 1) // pg
            vec = (ctypes.c_ubyte * npg)()
            if libc.mincore(a, n, vec) == 0:
                res += int((np.frombuffer(vec, np.uint8) & 1).sum())
                tot += npg
                nf += 1
            libc.munmap(a, n)
        finally:
            os.close(fd)
    out = {"files_sampled": nf, "pages": tot, "resident_frac": round(res / tot, 4) if tot else None}
    try:
        for line in open("/sys/fs/cgroup/memory.stat"):
            k, v = line.split()
            if k in ("file", "anon"):
                out[f"cgroup_{k}_GB"] = round(int(v) / 1e9, 2)
        mx = open("/sys/fs/cgroup/memory.max").read().strip()
        out["cgroup_memory_max_GB"] = None if mx == "max" else round(int(mx) / 1e9, 2)
    except (OSError, ValueError):
        pass
    return out


def locus_files(data: str) -> list:
    from mandalorion_amd import define

    tmp = os.path.join(data, "tmp_SS")
    return [os.path.join(tmp, r + ".psl") for r in define._roots(tmp)]


def shard_plan(data: str, world: int) -> list:
    """The driver's LPT plan (define.define_isoforms): loci per rank, for --check-launch."""
    from mandalorion_amd import define

    size_arr: list = []
    roots = define._roots(os.path.join(data, "tmp_SS"), size_array=size_arr)
    cost = define._size_costs(size_arr[0])
    owner = define._lpt_owner(cost, world)
    cnt = np.bincount(owner, minlength=world)
    load = np.bincount(owner, weights=cost, minlength=world)
    return [{"rank": k, "loci": int(cnt[k]), "cost_share": float(load[k] / max(load.sum(), 1e-9))} for k in range(world)]


def _prefix_sha(path: str, nbytes: int) -> str:
    h = hashlib.sha256()
    with open(path, "rb") as fh:
        left = nbytes
        while left > 0:
            blk = fh.read(min(left, 1 << 24))
            if not blk:
                break
            h.update(blk)
            left -= len(blk)
    return h.hexdigest()


def _headers_sha(path: str, limit: int = -1) -> str:
    """sha256 over the FASTA's first `limit` header lines (all: -1), newlines included."""
    h, n = hashlib.sha256(), 0
    with open(path, "rb") as fh:
        for line in fh:
            if line.startswith(b">"):
                if n == limit:
                    break
                h.update(line)
                n += 1
    return h.hexdigest()


def fullsize_check(data: str, key: str):
    """Both output files of the last step against the oracle's full-size hashes, and the clustering half
    (reads2isoforms.txt, the isoform header list) against the unmodified reference's own run on the same
    data (tests/golden/make_reference_fullsize.py: all loci, or a sorted-root prefix of them).  Returns
    (oracle ok, reference scope) or (None, None) without an entry; a mismatch fails the run."""
    if not os.path.exists(FULLSIZE_HASHES):
        return None, None
    ref = json.load(open(FULLSIZE_HASHES)).get(key)
    if ref is None:
        return None, None
    fa, r2 = os.path.join(data, "Isoform_Consensi.fasta"), os.path.join(data, "reads2isoforms.txt")
    got = {"isoform_consensi_sha256": sha(fa), "reads2isoforms_sha256": sha(r2)}
    ok = all(got[k] == ref[k] for k in got)
    if not ok:
        raise SystemExit(f"GPU D-module output of {key} differs from the oracle's full-size hashes: {got} vs "
                         f"{ {k: ref[k] for k in got} }")
    scope = None
    if "reference_reads2isoforms_sha256" in ref:
        hs = _headers_sha(fa)
        if got["reads2isoforms_sha256"] != ref["reference_reads2isoforms_sha256"] or hs != ref["reference_headers_sha256"]:
            raise SystemExit(f"GPU clustering of {key} differs from the reference's own run (reads2isoforms / headers)")
        scope = f"all {ref['loci']} loci"
    elif "reference_prefix" in ref:
        px = ref["reference_prefix"]
        if (_prefix_sha(r2, px["reads2isoforms_bytes"]) != px["reads2isoforms_sha256"]
                or _headers_sha(fa, px["isoforms"]) != px["headers_sha256"]):
            raise SystemExit(f"GPU clustering of {key} differs from the reference's own run on its first "
                             f"{px['loci']} loci (reads2isoforms prefix / headers)")
        scope = f"first {px['loci']} of {ref['loci']} loci (sorted roots)"
    return True, scope


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    if args.gpus != 1 and world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")
    wl = WORKLOADS[args.workload]
    n_loci = args.loci or wl["loci"]
    global SHARE
    if args.share > 1:
        if args.gpus != 1 or "WORLD_SIZE" in os.environ:
            raise SystemExit("--share runs one rank's load on one GPU (no launcher, --gpus 1)")
        SHARE = (0, args.share)
        args.no_cpu_baseline = True
    cores = host_cores()
    # host threads per rank: the usable cores per GPU of this node (a rank drives one GPU), at most 16
    threads = args.threads or max(2, min(16, cores["usable"] // max(1, local_world)))
    gen_threads = min(16, cores["usable"]) if rank == 0 else threads
    base = args.data_dir or os.environ.get("TMPDIR", "/tmp")
    data = os.path.join(base, f"mando_bench_{args.workload}_{n_loci}")
    os.makedirs(data, exist_ok=True)

    from mandalorion_amd import _lib

    comm = None
    if world > 1:
        from mandalorion_amd.comm import Comm

        comm = Comm.from_env(device=local, gpu=False if args.check_launch else None)
        if comm.backend != "rccl" and not args.check_launch:
            raise SystemExit(f"rank {rank}: {world} ranks need the RCCL transport, got {comm.backend!r}")
    n_gpus = comm.world if comm is not None else 1
    if rank == 0:
        tg = time.perf_counter()
        with heartbeat("synthetic data"):
            records = gen_data(data, wl, n_loci, gen_threads)
        log(f"data: {records} records in {data} ({time.perf_counter() - tg:.1f} s)")
    if comm is not None:
        comm.barrier()
    records = int(open(os.path.join(data, "records.txt")).read())

    if args.check_launch:
        plan = shard_plan(data, world)
        if comm is not None:
            comm.barrier()
            comm.close()
        if rank == 0:
            print(json.dumps({"check_launch": True, "n_gpus": n_gpus, "world": world,
                              "backend": comm.backend if comm is not None else "none", "records": records,
                              "ranks": plan, "host_cores": cores}), flush=True)
        return

    # CPU baseline first (rank 0 of a 1-GPU run): bounded sample, oracle orientation + POA on host threads
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu_threads = args.cpu_threads or cores["usable"]
        cpu, cpu_dir, cpu_hashes = cpu_baseline(data, min(args.cpu_loci, n_loci), cpu_threads)
        cpu.update(nproc=cores["nproc"], affinity=cores["affinity"], cgroup_quota=cores["cgroup_quota"])

    ctx = _lib.context(local)
    for k in range(args.warmup):
        tw = time.perf_counter()
        run_define(data, threads, local, comm)
        if rank == 0:
            log(f"warmup step {k}: {time.perf_counter() - tw:.3f} s")
    # page-cache residency of the locus text right before and after the timed steps (outside them)
    files = locus_files(data) if rank == 0 else []
    pc_before = page_cache_resident(files, stride=8) if rank == 0 else None
    if comm is not None:
        comm.barrier()
    ru0 = resource.getrusage(resource.RUSAGE_SELF)
    t0 = time.perf_counter()
    stats = []
    for k in range(args.steps):
        stats.append(run_define(data, threads, local, comm))
        if rank == 0:  # progress on stderr (a long run must not look idle); one line per step
            log(f"step {k}: {stats[-1]['t_total']:.3f} s")
    if comm is not None:
        comm.barrier()
    elapsed = time.perf_counter() - t0
    ru1 = resource.getrusage(resource.RUSAGE_SELF)
    host_cpu = (ru1.ru_utime - ru0.ru_utime + ru1.ru_stime - ru0.ru_stime) / max(1, args.steps)
    if comm is not None:
        elapsed = comm.max(elapsed)
    st = stats[-1]
    pc_after = page_cache_resident(files, stride=8) if rank == 0 else None

    # the whole output of the last timed step against the oracle's full-size hashes (rank 0 wrote it)
    full_parity, ref_scope = (fullsize_check(data, f"{args.workload}:{n_loci}") if rank == 0 and SHARE is None
                              else (None, None))
    if SHARE is not None:  # one rank's load: its own records
        records = stats[-1]["records"]

    # roofline of the dominant kernel (POA), from this rank's launches of the last timed step, per step:
    # algorithmic bytes = 1 B traceback per DP cell + each read once + each consensus once, over the POA
    # launches' HIP-event time (a batch's launch kinds run side by side: its time runs from the first
    # launch's start to the last one's end)
    la = st["poa_launches"]
    n_launch = sum(x["launches"] for x in la)
    alg = sum(x["cells"] + x["read_bytes"] + x["cons_bytes"] for x in la)
    k_ms = sum(x["kernel_ms"] for x in la)
    achieved = alg / (k_ms / 1e3) / 1e9 if k_ms > 0 else 0.0
    # HBM traffic per step from the PMC passes (tools/pmc_traffic.py: one step's POA dispatches), only when
    # they were measured on this workload, on the POA sources benchmarked now, under the same chunk plan,
    # chunk count and POA dispatch count as this step
    traffic, traffic_raw, pmc_note = None, None, "no PMC file"
    if os.path.exists(args.pmc_json):
        try:
            pm = json.load(open(args.pmc_json))
            if pm.get("workload") != f"{args.workload}:{n_loci}":
                pmc_note = f"PMC file is for {pm.get('workload')}"
            elif pm.get("poa_sources_sha256") != poa_sources_sha():
                pmc_note = "PMC file measured on other POA sources (dropped)"
            elif pm.get("plan") != plan_signature() or pm.get("chunks") != st.get("chunks"):
                pmc_note = (f"PMC file measured under another chunk plan ({pm.get('chunks')} chunks, "
                            f"{pm.get('plan')}; this step: {st.get('chunks')}) (dropped)")
            elif pm.get("poa_dispatches_per_step") != n_launch:
                pmc_note = (f"PMC file saw {pm.get('poa_dispatches_per_step')} POA dispatches per step, this "
                            f"step {n_launch} (dropped)")
            else:
                traffic = pm.get("hbm_bytes_per_step")
                traffic_raw = pm.get("hbm_bytes_per_step_raw")
                pmc_note = f"PMC passes of commit {pm.get('commit', '?')}, {n_launch} POA dispatches per step"
        except Exception as e:  # noqa: BLE001
            pmc_note = f"unreadable PMC file: {e}"

    # parity of the GPU path on the CPU baseline's sample (byte-identical output files)
    parity = None
    if cpu is not None:
        run_define(cpu_dir, threads, local)
        got = (sha(os.path.join(cpu_dir, "Isoform_Consensi.fasta")), sha(os.path.join(cpu_dir, "reads2isoforms.txt")))
        parity = got == cpu_hashes
        if not parity:
            raise SystemExit("GPU D-module output differs from the CPU restatement on the baseline sample")

    # the limiter from measurement: the HBM bytes the PMC passes saw per step over this step's POA launch
    # time, as a fraction of peak; well below peak the kernel is bound by instruction issue / latency (SQ
    # counters), not by HBM
    hbm_util = (traffic / (k_ms / 1e3) / 1e9 / HBM_PEAK_GBS) if traffic and k_ms > 0 else None
    bound = "hbm" if hbm_util is not None and hbm_util >= 0.6 else "issue"
    out = {
        "metric": "consensus reads/s (whole node): PSL records / wall s of Mando.py -M D",
        "value": records * args.steps / elapsed,
        "unit": "records/s",
        "n_gpus": n_gpus,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "int16",
        "data": "synthetic PSL loci (libmando_synth, seed 20250117): no real reads in the container",
        "config": {
            "workload": wl["text"] + (f" (loci overridden: {n_loci})" if args.loci else "")
                        + (f" -- rank 0's share of a {SHARE[1]}-rank LPT plan, run alone on one GPU" if SHARE else ""),
            "records": records,
            "loci": st["loci"],
            "isoforms": st["isoforms"],
            "poa_groups_rank0": st["poa_groups"],
            "poa_reads_rank0": st["poa_reads"],
            "parallelism": f"loci sharded over {n_gpus} GPU(s) (LPT on the DP-cost estimate), one all-gather "
                          f"({comm.backend if comm else 'none'}) to the writer on rank 0",
            "host_threads_per_rank": threads,
            # user + system CPU seconds of this rank's process per timed step (host waits sleep on the
            # device's completion signal, so this is the host work itself)
            "host_cpu_s_per_step_rank0": round(host_cpu, 2),
            "host_cores": cores,
            "phases_rank0_s": {k: round(st[k], 4) for k in ("t_ingest", "t_cluster", "t_orient", "t_assemble", "t_poa",
                                                             "t_merge", "t_write", "t_total") if k in st},
            "chunks": st.get("chunks"),
            "poa_kernel": {
                "launches": n_launch,
                "kernel_ms_total": k_ms,
                "dp_cells": sum(x["cells"] for x in la),
                "gcups": sum(x["cells"] for x in la) / (k_ms / 1e3) / 1e9 if k_ms > 0 else None,
                "reads_per_s": sum(x["reads"] for x in la) / (k_ms / 1e3) if k_ms > 0 else None,
            },
            "gpu_equals_cpu_on_sample": parity,
            "full_output_equals_oracle": full_parity,
            # reads2isoforms.txt and the isoform headers (clustering only) against the unmodified reference
            "clustering_equals_reference": ref_scope,
            # per timed step (rank 0): the D module's own wall time and its POA kernels' event time, so a
            # slow step shows where it lost its time
            "steps_s": [round(x["t_total"], 4) for x in stats],
            "steps_poa_kernel_ms": [round(sum(y["kernel_ms"] for y in x["poa_launches"]), 1) for x in stats],
            # the locus text's pages in the page cache (every 8th file) before / after the timed steps
            "page_cache": {"before": pc_before, "after": pc_after},
        },
        "roofline": {
            "bound": bound,
            "roofline": "hbm",
            "hbm_util": hbm_util,
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": traffic,
            "traffic_raw": traffic_raw,
            "traffic_unit": "HBM bytes per step (all POA dispatches of one step)",
            "achieved_unit": "algorithmic GB/s over the step's POA launch time",
            "poa_dispatches_per_step": n_launch,
            "traffic_source": pmc_note,
            "kernel": "poa_kernel",
            "note": "integer DP, no MFMA; the kernel is issue/latency-bound (SQ counters: DESIGN.md §3.1)",
        },
    }
    if cpu is not None:
        out["cpu_baseline"] = cpu
    if rank == 0:
        print(json.dumps(out), flush=True)
    if comm is not None:
        comm.close()
    ctx.close()


if __name__ == "__main__":
    main()
