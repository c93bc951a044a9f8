"""D module driver: the MI355X-native `defineIsoforms.py` (Mando.py -M D).

Same CLI and outputs as /root/reference/defineIsoforms.py:20-52 (`-i -p -c -g -w -m -W -n -j -u -d -a`);
writes <p>/Isoform_Consensi.fasta, <p>/reads2isoforms.txt and <p>/polyAWhiteList.bed.

Instead of one forked process per locus calling mappy + an `abpoa` subprocess per isoform
(defineIsoforms.py:130-153, SpliceDefineConsensus.py:876-931), the whole locus set goes through:
  1. clustering (libmando `mando_cluster_loci`, host C++ threads): peaks, isoform groups, RNG replay of
     every locus' draws and the determine_consensus subsample;
  2. orientation of every subsampled read against its isoform's first subsampled read
     (`mando_orient_batch`, HIP);
  3. the reference's per-isoform assembly logic (duplicate-primary rebinding, <=2 fallback, median
     length -> `-S`) on the host;
  4. one batched POA consensus over all remaining isoforms (`mando_poa_batch`, HIP);
  5. the ordered writer (sorted roots x IsoDict order, `Isoform{k}_{n}`).
Loci shard across ranks (torch.distributed, one process per GPU); the only exchange is the gather of
per-locus results to rank 0 for the writer.
"""
from __future__ import annotations

import argparse
import os
import sys
import time
from typing import Callable, Sequence

import numpy as np

from . import _lib, cluster, gtf

COMP = bytes.maketrans(b"ACGTNacgtn", b"TGCANtgcan")


def revcomp(s: str) -> str:
    """mappy.revcomp (ACGTN, either case)."""
    return s.encode().translate(COMP)[::-1].decode()


def gpu_orient(groups: Sequence[Sequence[str]], device: int = 0, max_hits: int = 4) -> list[list[list[int]]]:
    """Per group, per read: the strands (+1/-1) of its primary hits against the group's first read."""
    from . import orient

    return orient.orient_batch(groups, device=device, max_hits=max_hits)


def gpu_consensus(groups: Sequence[Sequence[str]], seeding: Sequence[bool], device: int = 0) -> list[str]:
    from . import poa

    if not groups:
        return []
    return poa.poa_consensus_batch(groups, seeding=seeding, device=device)


def _roots(out_tmp: str) -> list[str]:
    roots = set()
    for f in os.listdir(out_tmp):
        if os.path.isfile(os.path.join(out_tmp, f)) and ".psl" in f:
            root = f.split(".psl")[0]
            root.split("~")  # chrom~start~end (a '~' in a chrom name breaks the reference too)
            roots.add(root)
    return sorted(roots, key=lambda x: (x.split("~")[0], int(x.split("~")[1])))


def assemble(res: cluster.ClusterResult, iso_idx: Sequence[int], strands: list[list[list[int]]]):
    """determine_consensus (SpliceDefineConsensus.py:876-931) minus the POA call, per isoform.

    Returns (direct, poa_groups, poa_seeding, poa_owner): direct[i] is the consensus when no POA run
    is needed (<=2 oriented sequences), else None and the isoform's group is in poa_groups."""
    direct: list[str | None] = []
    groups, seeding, owner, firsts = [], [], [], []
    for gi, i in enumerate(iso_idx):
        sub = res.subsample(i)
        seqs, lens = [], []
        for r, st in zip(sub, strands[gi]):
            s = res.seq(int(r))
            lens.append(len(s))
            for strand in st:  # every primary hit writes the (re-bound) sequence once (SDC:902-907)
                if strand == -1:
                    s = revcomp(s)
                seqs.append(s)
        if not seqs:
            raise IndexError(f"isoform {i}: no subsampled read maps to the first one "
                             "(the reference raises IndexError at SpliceDefineConsensus.py:912)")
        if len(seqs) <= 2:
            direct.append(seqs[0])
        else:
            direct.append(None)
            groups.append(seqs)
            seeding.append(bool(np.median(lens) >= 8000))
            owner.append(gi)
            firsts.append(seqs[0])
    return direct, groups, seeding, owner, firsts


def define_isoforms(path: str, cutoff: float = 0.1, genome_file: str = "None", splice_site_width: int = 1,
                    minimum_read_count: int = 2, white_list_polyA: Sequence[str] = ("0",), threads: int = 0,
                    junctions: str = "gtag,gcag,atac,ctac,ctgc,gtat", upstream_buffer: int = 10,
                    downstream_buffer: int = 50, seed: int = 0, device: int = 0,
                    orient_fn: Callable | None = None, consensus_fn: Callable | None = None,
                    rank: int = 0, world: int = 1, comm=None, verbose: bool = False) -> dict:
    """Runs the D module on <path>/tmp_SS/*.psl.  orient_fn / consensus_fn default to the HIP path."""
    t0 = time.perf_counter()
    orient_fn = orient_fn or (lambda g: gpu_orient(g, device=device))
    consensus_fn = consensus_fn or (lambda g, s: gpu_consensus(g, s, device=device))
    out_path = path + "/"
    out_tmp = out_path + "/tmp_SS"
    wl = list(white_list_polyA)
    left, right, poly = {}, {}, []
    if genome_file != "None" and (genome_file.endswith(".gtf.gz") or genome_file.endswith(".gtf")):
        _, left, right, poly = gtf.parse_genome(genome_file, wl)
    if rank == 0:
        gtf.write_polya_bed(out_path + "/polyAWhiteList.bed", poly, wl)
    roots = _roots(out_tmp)
    # shard loci over ranks: LPT on file size (cost ~ reads x length), results regathered in root order
    mine = list(range(len(roots)))
    if world > 1:
        sizes = [os.path.getsize(os.path.join(out_tmp, r + ".psl")) for r in roots]
        load = [0] * world
        owner = [0] * len(roots)
        for i in sorted(range(len(roots)), key=lambda i: -sizes[i]):
            k = int(np.argmin(load))
            owner[i] = k
            load[k] += sizes[i]
        mine = [i for i in range(len(roots)) if owner[i] == rank]
    my_roots = [roots[i] for i in mine]
    chroms = [r.split("~")[0] for r in my_roots]
    ann = [gtf.locus_bounds(left, right, r.split("~")[0], int(r.split("~")[1]), int(r.split("~")[2]))
           for r in my_roots]
    t1 = time.perf_counter()
    res = cluster.cluster_loci([os.path.join(out_tmp, r + ".psl") for r in my_roots], chroms, ann=ann,
                               cutoff=cutoff, splice_site_width=splice_site_width,
                               minimum_read_count=minimum_read_count, upstream_buffer=upstream_buffer,
                               downstream_buffer=downstream_buffer, junctions=junctions, seed=seed,
                               threads=threads)
    bad = np.nonzero(res.locus_status != 0)[0]
    if len(bad):
        i = int(bad[0])
        raise RuntimeError(f"locus {my_roots[i]}: {cluster.STATUS.get(int(res.locus_status[i]), res.locus_status[i])} "
                           "(the reference's locus worker raises here)")
    t2 = time.perf_counter()
    n_iso = res.n_isoforms
    iso_idx = list(range(n_iso))
    og = [[res.seq(int(r)) for r in res.subsample(i)] for i in iso_idx]
    strands = orient_fn(og)
    t3 = time.perf_counter()
    direct, groups, seeding, owner, firsts = assemble(res, iso_idx, strands)
    cons = consensus_fn(groups, seeding)
    for k, gi in enumerate(owner):
        direct[gi] = cons[k] if cons[k] else firsts[k]
    t4 = time.perf_counter()
    # per-locus records for the writer: (root index, [(consensus, [names])...])
    per_locus: dict[int, list] = {mine[li]: [] for li in range(len(my_roots))}
    for i in iso_idx:
        li = int(res.iso_locus[i])
        per_locus[mine[li]].append((direct[i], [res.name(int(r)) for r in res.members(i)]))
    if world > 1:
        per_locus = _gather(per_locus, rank, world, comm)
    stats = {"loci": len(roots), "isoforms": n_iso, "poa_groups": len(groups),
             "records": int(res.n_records), "poa_reads": int(sum(len(g) for g in groups)),
             "t_ingest": t1 - t0, "t_cluster": t2 - t1, "t_orient": t3 - t2, "t_poa": t4 - t3}
    if rank == 0:
        counter = 0
        with open(out_path + "/Isoform_Consensi.fasta", "w") as out, open(out_path + "/reads2isoforms.txt", "w") as r2i:
            for ri in range(len(roots)):
                for consensus, names in per_locus.get(ri, []):
                    counter += 1
                    nm = "Isoform" + str(counter) + "_" + str(len(names))
                    out.write(">%s\n%s\n" % (nm, consensus))
                    for n in names:
                        r2i.write("%s\t%s\n" % (n, nm))
        stats["written_isoforms"] = counter
    stats["t_total"] = time.perf_counter() - t0
    res.close()
    if verbose and rank == 0:
        print("\t" + " ".join(f"{k}={v:.3f}" if isinstance(v, float) else f"{k}={v}" for k, v in stats.items()))
    return stats


def _gather(per_locus: dict, rank: int, world: int, comm) -> dict:
    """Reassembly on rank 0: one all-gather of byte counts, one of padded byte buffers (RCCL over xGMI
    with the nccl backend, gloo on CPU)."""
    import torch
    import torch.distributed as dist

    blob = _serialize(per_locus)
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
    n = torch.tensor([len(blob)], dtype=torch.int64, device=dev)
    ns = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(ns, n)
    mx = int(max(int(x.item()) for x in ns))
    buf = torch.zeros(mx, dtype=torch.uint8, device=dev)
    if blob:
        buf[:len(blob)] = torch.frombuffer(bytearray(blob), dtype=torch.uint8).to(dev)
    bufs = [torch.zeros_like(buf) for _ in range(world)]
    dist.all_gather(bufs, buf)
    merged: dict[int, list] = {}
    if rank == 0:
        for k in range(world):
            raw = bytes(bufs[k][: int(ns[k].item())].cpu().numpy())
            merged.update(_deserialize(raw))
    return merged


def _serialize(per_locus: dict) -> bytes:
    parts = []
    for ri, isos in per_locus.items():
        parts.append(f"L\t{ri}\t{len(isos)}\n")
        for consensus, names in isos:
            parts.append(f"I\t{consensus}\t{len(names)}\n")
            parts.append("\t".join(names) + "\n")
    return "".join(parts).encode()


def _deserialize(raw: bytes) -> dict:
    out: dict[int, list] = {}
    lines = raw.decode().split("\n")
    i = 0
    while i < len(lines) and lines[i]:
        _, ri, niso = lines[i].split("\t")
        i += 1
        isos = []
        for _ in range(int(niso)):
            _, consensus, nn = lines[i].split("\t")
            names = lines[i + 1].split("\t") if int(nn) else []
            isos.append((consensus, names))
            i += 2
        out[int(ri)] = isos
    return out


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
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        import torch
        import torch.distributed as dist

        if torch.cuda.is_available():
            torch.cuda.set_device(a.device)
            dist.init_process_group("nccl", device_id=torch.device("cuda", a.device))
        else:
            dist.init_process_group("gloo")
    define_isoforms(a.path, cutoff=float(a.cutoff), genome_file=a.genome_file, splice_site_width=int(a.splice_site_width),
                    minimum_read_count=int(a.minimum_read_count), white_list_polyA=a.white_list_polyA.split(","),
                    threads=int(a.numThreads), junctions=a.junctions, upstream_buffer=int(a.upstream_buffer),
                    downstream_buffer=int(a.downstream_buffer), seed=a.seed, device=a.device, rank=rank,
                    world=world, verbose=True)
    if world > 1:
        import torch.distributed as dist

        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
