"""`Mando.py`-compatible entry point of this build (python -m mandalorion_amd.mando ... or ./Mando.py).

Keeps the reference's command-line surface (/root/reference/Mando.py:22-205) so a pipeline that calls
`Mando.py -M D ...` can switch over unchanged.  Only the D module (defining isoforms) is built here:
it runs mandalorion_amd.define (clustering, orientation and POA consensus as HIP kernels on the GPU;
the host reads the locus files and writes the outputs) with exactly the arguments Mando.py passes to defineIsoforms.py (Mando.py:382-399).  Module P
(SAM -> PSL, clean_psl, sort + locus split: the D module's input) runs natively (mandalorion_amd.psl);
so do modules F (isoform filters, with minimap2 as the external aligner of the consensi or an existing
tmp/Isoforms.aligned.out.sam) and Q (quantification) (mandalorion_amd.modules).  Module A (read
alignment) and F's gene grouping (groupIsoforms.py) are outside this build's scope and are
reported and skipped.  Without a SAM, P starts from an existing clean PSL.
"""
from __future__ import annotations

import argparse
import os
import sys
from time import localtime, strftime

VERSION = "mandalorion_amd 0.1.0 (D module on MI355X; CLI of Mandalorion v4.2.0)"


def parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(description="Mandalorion isoform identification (MI355X D module)")
    ap.add_argument("-p", "--path", type=str, default=".", help="output directory")
    ap.add_argument("-u", "--upstream_buffer", type=str, default="10")
    ap.add_argument("-d", "--downstream_buffer", type=str, default="50")
    ap.add_argument("-g", "--genome_annotation", type=str, default="None", help="GTF (annotated splice sites)")
    ap.add_argument("-G", "--genome_sequence", type=str)
    ap.add_argument("-r", "--minimum_ratio", type=str, default="0.01")
    ap.add_argument("-i", "--minimum_internal_ratio", type=str, default="1")
    ap.add_argument("-R", "--minimum_reads", type=str, default="3")
    ap.add_argument("-f", "--Consensus_reads", type=str, help="reads: file, comma list, or .fofn")
    ap.add_argument("-O", "--overhangs", type=str, default="0,40,0,40")
    ap.add_argument("-t", "--minimap2_threads", type=str, default="8")
    ap.add_argument("-I", "--minimum_isoform_length", type=str, default="200")
    ap.add_argument("-n", "--minimum_feature_count", type=str, default="2")
    ap.add_argument("-w", "--splice_site_window", type=str, default="1")
    ap.add_argument("-A", "--Acutoff", type=str, default="0.5")
    ap.add_argument("-W", "--white_list_polyA", type=str, default="0")
    ap.add_argument("-m", "--multi_exon_only", default="0", action="store_const", const="1")
    ap.add_argument("-j", "--junctions", default="gtag,gcag,atac,ctac,ctgc,gtat", type=str)
    ap.add_argument("-M", "--Modules", default="APDFQ")
    ap.add_argument("-P", "--pacbio", default=False, action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--mm2_path", default=None, type=str, help=argparse.SUPPRESS)
    ap.add_argument("--seed", type=int, default=int(os.environ.get("MANDO_RNG_SEED", "0")),
                    help="numpy RNG state every locus starts from (the reference's parent process state)")
    ap.add_argument("-v", "--version", action="version", version=VERSION)
    return ap


def main(argv: list[str] | None = None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    ap = parser()
    if not argv:
        ap.print_help()
        return 0
    a = ap.parse_args(argv)
    path = a.path + "/"
    temp_path = path + "/tmp/"
    files = a.Consensus_reads or ""
    if ".fofn" in files:
        fasta_list = [l.strip() for l in open(files)]
    else:
        fasta_list = files.split(",") if files else []
    os.makedirs(path, exist_ok=True)
    with open(path + "/Mando.log", "a") as log:
        log.write(f'\nMandalorion "{VERSION}" was run on {strftime("%Y-%m-%d %H:%M:%S", localtime())}\n'
                  f"with the following parameters\n{str(a).replace('Namespace(', '').replace(')', '')}\n")
    os.makedirs(temp_path, exist_ok=True)
    # The reference runs its modules in a fixed order whatever the order of the -M string
    # (Mando.py:270-475).  Under a multi-rank launch (WORLD_SIZE > 1) only the D module is sharded:
    # P, F and Q run on rank 0 alone, and every rank waits for P before D reads tmp_SS.
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    comm = None
    if world > 1:
        from .comm import Comm

        comm = Comm.from_env()
    try:
        _run_modules(a, path, temp_path, fasta_list, comm, rank)
    finally:
        if comm is not None:
            comm.close()
    return 0


def _run_modules(a, path: str, temp_path: str, fasta_list: list, comm, rank: int) -> None:
    for mod in "APDFQ":
        if mod not in a.Modules:
            continue
        if mod == "D" and comm is not None:
            comm.barrier()  # module P (rank 0) has written tmp_SS
        if rank != 0 and mod != "D":
            continue
        if mod == "P":
            # module P (Mando.py:323-358): SAM -> PSL (emtrey -m), clean_psl, sort + locus split, all native
            import shutil

            from . import psl

            sam = temp_path + "/mm2Alignments.sam"
            clean = temp_path + "/mm2Alignments.clean.psl"
            if os.path.exists(sam) and os.path.getsize(sam) > 0:
                print("\tconverting sam output to psl format")
                psl.sam_to_psl(sam, temp_path + "/mm2Alignments.psl", mando=True, threads=int(a.minimap2_threads))
                print("\tcleaning psl file of small Indels")
                psl.clean_psl(temp_path + "/mm2Alignments.psl", clean, True)
            elif not os.path.exists(clean) or os.path.getsize(clean) == 0:
                print("\tno or empty SAM file was provided. File conversions and parsing not performed")
                continue
            print("\tsorting clean psl file and splitting it into loci")
            shutil.rmtree(temp_path + "/tmp_SS", ignore_errors=True)
            nrec, nloc = psl.split_loci(clean, temp_path + "/tmp_SS", sort_lines=True,
                                        sorted_out=temp_path + "/mm2Alignments.clean.sorted.psl")
            print(f"\t\tsplit {nrec} psl entries into {nloc} loci")
            continue
        if mod == "F":
            # module F (Mando.py:404-470): filterIsoforms natively; the consensi's alignment is minimap2's
            # (--mm2_path) or an existing tmp/Isoforms.aligned.out.sam
            import shutil

            from . import modules, psl

            iso = temp_path + "/Isoform_Consensi.fasta"
            ok = os.path.exists(iso) and os.path.getsize(iso) > 0
            if not ok:
                print("\tisoforms fasta missing or empty")
            if not a.genome_sequence or not os.path.exists(a.genome_sequence) or os.path.getsize(a.genome_sequence) == 0:
                print("\tgenome sequence fasta missing or empty")
                ok = False
            if not ok:
                print("\tone or more input files missing or empty. Isoforms not filtered")
                continue
            p = modules.FilterParams.default()
            p.minimum_ratio = float(a.minimum_ratio)
            p.minimum_reads = float(a.minimum_reads)
            p.internal_ratio = float(a.minimum_internal_ratio)
            p.Acutoff = float(a.Acutoff)
            for i, v in enumerate(a.overhangs.split(",")):
                p.overhangs[i] = int(v)
            p.splice_window = int(a.splice_site_window)
            p.downstream_buffer = int(a.downstream_buffer)
            p.minimum_isoform_length = int(a.minimum_isoform_length)
            p.multi_exon_only = int(a.multi_exon_only)
            p.threads = int(a.minimap2_threads)
            n = modules.module_f(temp_path, iso, a.genome_sequence, p, minimap2=a.mm2_path,
                                 threads=int(a.minimap2_threads))
            print(f"\t{n} isoforms kept")
            srt = temp_path + "/Isoforms.sorted.psl"
            psl.split_loci(temp_path + "/Isoforms.filtered.clean.psl", temp_path + "/tmp_iso_split", sort_lines=True,
                           sorted_out=srt)
            shutil.rmtree(temp_path + "/tmp_iso_split", ignore_errors=True)
            from . import genes

            print("\tgrouping isoforms and assigning them to genes (if annotation is provided)")
            genes.group_isoforms(srt, temp_path + "/Isoforms.filtered.clean.genes", a.genome_annotation)
            for f in os.listdir(temp_path):
                if f.startswith("Isoforms.filtered."):
                    shutil.copy(os.path.join(temp_path, f), path)
            continue
        if mod == "Q":
            # module Q (Mando.py:474-491): assignReadsToIsoforms natively
            import shutil

            from . import modules

            modules.quantify(temp_path, fasta_list)
            for f in ("Isoforms.filtered.clean.quant", "Isoforms.filtered.clean.tpm"):
                shutil.copy(temp_path + "/" + f, path)
            continue
        if mod != "D":
            print(f"\tmodule {mod}: not part of this build (D module only), skipped")
            continue
        print("\n      Module D - defining isoforms (MI355X)\n")
        clean_sorted = temp_path + "/mm2Alignments.clean.sorted.psl"
        ok = True
        if not os.path.exists(clean_sorted) or os.path.getsize(clean_sorted) == 0:
            print("\tclean sorted psl file missing or empty")
            ok = False
        for f in fasta_list:
            if not os.path.exists(f) or os.path.getsize(f) == 0:
                print("\t", f, "missing or empty")
                ok = False
        if not ok:
            continue
        from . import define

        local = int(os.environ.get("LOCAL_RANK", "0"))
        st = define.define_isoforms(temp_path, cutoff=0.1, genome_file=a.genome_annotation,
                               splice_site_width=int(a.splice_site_window),
                               minimum_read_count=int(a.minimum_feature_count),
                               white_list_polyA=a.white_list_polyA.split(","), threads=int(a.minimap2_threads),
                               junctions=a.junctions, upstream_buffer=int(a.upstream_buffer),
                               downstream_buffer=int(a.downstream_buffer), seed=a.seed, device=local, comm=comm,
                               verbose=True)
        if rank == 0:
            # Mando.py:400: the read -> isoform table is also kept next to the outputs
            import json
            import shutil

            shutil.copy(temp_path + "/reads2isoforms.txt", path + "Mando_isoforms.read_stat.txt")
            # this build's metrics line next to Mando.log (one JSON object per run)
            with open(path + "/Mando.metrics.jsonl", "a") as fh:
                fh.write(json.dumps(dict(define.metrics(st, comm.world if comm is not None else 1),
                                         time=strftime("%Y-%m-%d %H:%M:%S", localtime()))) + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
