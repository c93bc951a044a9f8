#!/usr/bin/env python3
"""Benchmark of the D-module hot path: batched POA consensus on MI355X (libmando, HIP/gfx950).

Workload (BASELINE.json configs[2], "1M synthetic 3 kb R2C2 reads over 20k loci"): per rank, 20,000
isoform read groups x 50 reads, templates uniform 2.7-3.3 kb, R2C2 error model (synthetic, seed
20250117 + rank), already oriented — i.e. exactly what determine_consensus hands abPOA.  One step =
one mando_poa_batch_device call over all groups with every input resident in HBM, plus (N>1) the
RCCL all-gather that reassembles the consensus FASTA on rank 0.  Loci shard across ranks (weak
scaling: every rank gets its own 1M-read shard), no data-path collective besides the reassembly.

Prints ONE JSON line (rank 0).  metric/unit follow BASELINE.json: consensus reads/s (whole node).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import multiprocessing as mp
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X spec, MI355X_MICROARCH.md "Chip-level parameters"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--groups", type=int, default=20000)
    ap.add_argument("--depth", type=int, default=50)
    ap.add_argument("--len-lo", type=int, default=2700)
    ap.add_argument("--len-hi", type=int, default=3300)
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--cpu-procs", type=int, default=0, help="0 = min(16, cpu_count)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--pmc-json", default=os.path.join(ROOT, "profiles", "pmc_latest.json"))
    ap.add_argument("--e2e-loci", type=int, default=2000,
                    help="also time the whole D module (define_isoforms: PSL files -> FASTA) on this many "
                         "synthetic 50-read loci; 0 = skip (reported as d_module, never as value)")
    return ap.parse_args()


_ENC = np.full(256, 4, dtype=np.uint8)
for _c, _v in zip(b"ACGTacgt", (0, 1, 2, 3, 0, 1, 2, 3)):
    _ENC[_c] = _v


def lpt_order(seq_off, grp_off):
    """Groups sorted by estimated DP work (reads x first-read length), largest first."""
    lens = np.diff(seq_off)
    first = lens[grp_off[:-1]]
    tot = np.add.reduceat(lens, grp_off[:-1]) if len(lens) else np.zeros(0)
    return np.argsort(-(tot - first).astype(np.float64) * first, kind="stable")


def reorder(seqs, seq_off, grp_off, order):
    """Repack groups in `order` (so the device processes the heaviest groups first)."""
    parts, offs, goff = [], [0], [0]
    total = 0
    for g in order:
        a, b = grp_off[g], grp_off[g + 1]
        s0, s1 = seq_off[a], seq_off[b]
        parts.append(seqs[s0:s1])
        offs.extend((seq_off[a + 1:b + 1] - s0 + total).tolist())
        total += s1 - s0
        goff.append(goff[-1] + (b - a))
    return np.concatenate(parts), np.asarray(offs, dtype=np.int64), np.asarray(goff, dtype=np.int64)


def _cpu_worker(args):
    groups, deadline = args
    from oracle import poa as opoa

    done_reads = 0
    done_groups = 0
    t0 = time.perf_counter()
    for g in groups:
        if time.perf_counter() > deadline:
            break
        opoa.consensus_batch([g])
        done_reads += len(g)
        done_groups += 1
    return done_reads, done_groups, time.perf_counter() - t0


def _cpu_init():
    from oracle import poa as opoa

    opoa.load()


def cpu_baseline(seqs, seq_off, grp_off, seconds, procs):
    """oracle/poa_ref.c (C restatement of abPOA, 1 thread per process) on a time-bounded sample.

    Runs before the GPU is initialised, in `spawn` workers (no inherited HIP state); each process gets
    far more groups than it can finish (~0.2 s per 50x3kb group) and stops at the shared deadline."""
    from mandalorion_amd import synth

    n_groups = len(grp_off) - 1
    per = max(8, int(seconds * 12))
    want = min(n_groups, procs * per)
    pick = list(range(0, n_groups, max(1, n_groups // want)))[:want]  # evenly strided sample
    groups = synth.unpack_groups(seqs, seq_off, grp_off, pick)
    chunks = [groups[i::procs] for i in range(procs)]
    ctx = mp.get_context("spawn")
    with ctx.Pool(procs, initializer=_cpu_init) as pool:
        pool.map(_cpu_init_probe, range(procs))  # workers up and the oracle loaded before the clock
        t0 = time.perf_counter()
        deadline = t0 + seconds
        res = pool.map(_cpu_worker, [(c, deadline) for c in chunks])
        wall = time.perf_counter() - t0
    reads = sum(r[0] for r in res)
    ngr = sum(r[1] for r in res)
    return {
        "value": reads / wall if wall > 0 else 0.0,
        "unit": "reads/s",
        "cores": procs,
        "kind": "port",
        "sample": f"{ngr} groups x {groups[0] and len(groups[0])} reads of this workload through oracle/poa_ref.c "
                  f"(C restatement of abPOA v1.4.1, scalar), {procs} processes, {wall:.1f} s wall",
    }


def d_module_e2e(n_loci, device):
    """Whole D module (mandalorion_amd.define.define_isoforms, i.e. `Mando.py -M D`): locus PSL files on
    disk -> clustering (host C++) -> orientation + POA (GPU) -> Isoform_Consensi.fasta.  Reported as
    PSL records / wall second, the BASELINE.md end-to-end metric, on a config-3-shaped sample."""
    import shutil
    import tempfile

    from mandalorion_amd import define, synth

    d = tempfile.mkdtemp(prefix="mando_e2e_", dir=os.environ.get("TMPDIR", "/tmp"))
    try:
        n = synth.write_loci(os.path.join(d, "tmp_SS"), n_loci, threads=16)
        define.define_isoforms(d, threads=16, device=device)  # warm (context, kernels, page cache)
        t0 = time.perf_counter()
        st = define.define_isoforms(d, threads=16, device=device)
        wall = time.perf_counter() - t0
    finally:
        shutil.rmtree(d, ignore_errors=True)
    return {"records": n, "loci": st["loci"], "isoforms": st["isoforms"], "poa_groups": st["poa_groups"],
            "wall_s": wall, "reads_per_s": n / wall, "t_cluster": st["t_cluster"], "t_orient": st["t_orient"],
            "t_poa": st["t_poa"], "host_threads": 16,
            "input": f"{n_loci} synthetic loci x 50 R2C2 reads (5-12 exons of 150-400 nt), PSL files on disk"}


def _cpu_init_probe(_):
    return os.getpid()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    from mandalorion_amd import synth

    seqs, seq_off, grp_off = synth.fast_groups(args.groups, (args.len_lo, args.len_hi),
                                               (args.depth, args.depth), seed=synth.DATA_SEED + rank,
                                               threads=16)
    # CPU baseline first, on rank 0 of a 1-GPU run, before anything touches the GPU
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        procs = args.cpu_procs or min(16, os.cpu_count() or 1)
        cpu = cpu_baseline(seqs, seq_off, grp_off, args.cpu_seconds, procs)
    import torch

    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)

    from mandalorion_amd import _lib

    ctx = _lib.context(local)
    order = lpt_order(seq_off, grp_off)
    seqs, seq_off, grp_off = reorder(seqs, seq_off, grp_off, order)
    n_groups = len(grp_off) - 1
    n_reads = len(seq_off) - 1
    lens = np.diff(seq_off)
    max_len = int(lens.max())
    gsum = np.add.reduceat(lens, grp_off[:-1])
    ccap = np.zeros(n_groups + 1, dtype=np.int64)
    np.cumsum(2 * np.maximum.reduceat(lens, grp_off[:-1]) + 256, out=ccap[1:])

    d_seq = torch.from_numpy(_ENC[seqs]).to(dev)
    d_seq_off = torch.from_numpy(seq_off).to(dev)
    d_grp_off = torch.from_numpy(grp_off).to(dev)
    d_cons_off = torch.from_numpy(ccap).to(dev)
    d_cons = torch.zeros(int(ccap[-1]), dtype=torch.uint8, device=dev)
    d_cons_len = torch.zeros(n_groups, dtype=torch.int32, device=dev)
    d_cells = torch.zeros(n_groups, dtype=torch.int64, device=dev)
    d_status = torch.full((n_groups,), 99, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    p = _lib.PoaParams.defaults()

    def step():
        _lib.check(ctx.lib.mando_poa_batch_device(
            ctx.handle, ctypes.byref(p), d_seq.data_ptr(), d_seq_off.data_ptr(), d_grp_off.data_ptr(),
            n_groups, max_len, int(gsum.max()), d_cons.data_ptr(), d_cons_off.data_ptr(),
            d_cons_len.data_ptr(), d_cells.data_ptr(), d_status.data_ptr()))
        ctx.sync()
        if dist is not None:  # reassembly of the consensus FASTA on rank 0 (RCCL over xGMI)
            lens_all = [torch.empty_like(d_cons_len) for _ in range(world)]
            dist.all_gather(lens_all, d_cons_len)
            cons_all = [torch.empty_like(d_cons) for _ in range(world)]
            dist.all_gather(cons_all, d_cons)
        return ctx.last_kernel_ms()

    for _ in range(args.warmup):
        step()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    kms = [step() for _ in range(args.steps)]
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    status = d_status.cpu().numpy()
    if (status != 0).any():
        raise SystemExit(f"rank {rank}: {int((status != 0).sum())} groups failed (status {np.unique(status)})")
    cells = d_cells.cpu().numpy()
    clen = d_cons_len.cpu().numpy().astype(np.int64)
    # spot parity check of two groups against the CPU restatement (full parity: tests/test_poa_gpu.py)
    if rank == 0:
        from oracle import poa as opoa

        pick = [n_groups - 1, n_groups // 2]
        want = opoa.consensus_batch(synth.unpack_groups(seqs, seq_off, grp_off, pick))
        raw = d_cons.cpu().numpy()
        got = [bytes(raw[ccap[g]:ccap[g] + clen[g]]).translate(bytes.maketrans(b"\0\1\2\3\4", b"ACGTN")).decode()
               for g in pick]
        if got != want:
            raise SystemExit("GPU consensus differs from the CPU restatement on the spot check")

    # roofline: algorithmic bytes per launch = 1 B traceback per DP cell + each read once + consensus
    alg_bytes = float(cells.sum() + lens.sum() + clen.sum())
    kernel_s = float(np.mean(kms)) / 1e3
    achieved = alg_bytes / kernel_s / 1e9
    traffic = None
    if os.path.exists(args.pmc_json):
        try:
            pm = json.load(open(args.pmc_json))
            if pm.get("workload") == f"{args.groups}x{args.depth}x{args.len_lo}-{args.len_hi}":
                traffic = pm.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None
    out = {
        "metric": "consensus reads/s (whole node)",
        "value": world * n_reads * args.steps / elapsed,
        "unit": "reads/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int16",
        "data": "synthetic R2C2-shaped read groups (seed 20250117+rank), oriented, inputs resident in HBM",
        "config": {
            "workload": f"config3: {n_groups} isoform groups x {args.depth} reads x {args.len_lo}-{args.len_hi} nt "
                        f"per GPU ({n_reads} reads), abPOA -M 5 -r 0 semantics",
            "groups_per_gpu": n_groups,
            "reads_per_gpu": n_reads,
            "parallelism": f"loci sharded over {world} GPU(s), RCCL all-gather reassembly",
            "dp_cells_per_launch": int(cells.sum()),
            "kernel_ms": float(np.mean(kms)),
            "gcups": float(cells.sum()) / kernel_s / 1e9,
        },
        "roofline": {
            "bound": "hbm",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": traffic,
        },
    }
    if cpu is not None:
        out["cpu_baseline"] = cpu
    if rank == 0 and world == 1 and args.e2e_loci > 0:
        out["d_module"] = d_module_e2e(args.e2e_loci, local)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
