#!/usr/bin/env python3
"""Generates tests/golden/gene_vectors.json: the reference's gene grouping (run here only).

Input (`make_input`, numpy default_rng, no reference code): a synthetic GTF (genes on both strands
and three chromosomes; even- and odd-start exons; overlapping and nested genes; gene_name present or
absent; one gene_id with exons on two chromosomes; comment, gene and transcript lines) and a sorted
24-column PSL of isoforms (overlapping isoform chains that merge into one locus, isolated isoforms,
isoforms outside every gene, multi-block isoforms).  Two annotations: the GTF, and 'None'.
Reference path (Mando.py:458-469): `python3 groupIsoforms.py -i Isoforms.sorted.psl -o out -g gtf`,
PYTHONHASHSEED=0.  Stored: the input files and the output lines, the overlap column split into a
sorted list (the reference joins a Python set, whose order depends on the hash seed).
Nothing of the reference is copied.
"""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/groupIsoforms.py"


def make_input(seed=20251016):
    rng = np.random.default_rng(seed)
    gtf, psl = ["#!genome-build synthetic"], []
    gid = 0
    for chrom in ("chr1", "chr2", "chrX"):
        for strand in "+-":
            pos = int(rng.integers(100, 400))
            for _ in range(6):
                gid += 1
                nex = int(rng.integers(1, 5))
                exons, p = [], pos
                for _ in range(nex):
                    ln = int(rng.integers(40, 300))
                    exons.append((p, p + ln))
                    p += ln + int(rng.integers(50, 400))
                attrs = f'gene_id "G{gid}"; transcript_id "T{gid}";'
                if gid % 3:
                    attrs += f' gene_name "N{gid}";'
                gtf.append("\t".join([chrom, "syn", "gene", str(exons[0][0] + 1), str(exons[-1][1]), ".", strand, ".",
                                      attrs]))
                for s, e in exons:
                    gtf.append("\t".join([chrom, "syn", "exon", str(s + 1), str(e), ".", strand, ".", attrs]))
                # isoforms over this gene: 0-3, some shifted so that neighbours chain into one locus
                for k in range(int(rng.integers(0, 4))):
                    sh = int(rng.integers(-60, 60))
                    blocks = [(max(0, s + sh + int(rng.integers(-20, 20))), e + sh) for s, e in exons]
                    blocks = [(s, max(s + 10, e)) for s, e in blocks]
                    if k == 2:
                        blocks = blocks[:1]
                    psl.append((chrom, strand, blocks))
                # genes overlap their predecessor half the time (nested / shared bases)
                pos = p + (int(rng.integers(-800, -100)) if rng.random() < 0.5 else int(rng.integers(200, 2000)))
                pos = max(pos, 10)
            # an isoform far away from every gene
            psl.append((chrom, strand, [(pos + 50000, pos + 50300), (pos + 50500, pos + 50700)]))
    # one gene_id with exons on two chromosomes (first exon line's chromosome wins)
    attrs = 'gene_id "GSPLIT"; gene_name "SPLIT";'
    gtf.append("\t".join(["chr2", "syn", "exon", "201", "400", ".", "+", ".", attrs]))
    gtf.append("\t".join(["chr1", "syn", "exon", "150", "600", ".", "+", ".", attrs]))
    rows = []
    for i, (chrom, strand, blocks) in enumerate(psl):
        blocks = sorted(blocks)
        merged = []
        for s, e in blocks:
            if merged and s <= merged[-1][1]:
                merged[-1] = (merged[-1][0], max(merged[-1][1], e))
            else:
                merged.append((s, e))
        size = sum(e - s for s, e in merged)
        qs, q = [], 0
        for s, e in merged:
            qs.append(q)
            q += e - s
        rows.append([str(size), "0", "0", "0", "0", "0", "0", "0", strand, f"Isoform{i}_{3 + i % 7}", str(size), "0",
                     str(size), chrom, "1000000", str(merged[0][0]), str(merged[-1][1]), str(len(merged)),
                     "".join(f"{e - s}," for s, e in merged), "".join(f"{x}," for x in qs),
                     "".join(f"{s}," for s, _ in merged), "0.99", "cs", "ACGT"])
    rows.sort(key=lambda a: (a[13], int(a[15]), "\t".join(a)))
    return "\n".join(gtf) + "\n", "".join("\t".join(a) + "\n" for a in rows)


def run_reference(gtf_text, psl_text, annotated):
    with tempfile.TemporaryDirectory() as d:
        g = os.path.join(d, "ann.gtf")
        p = os.path.join(d, "Isoforms.sorted.psl")
        o = os.path.join(d, "genes.txt")
        open(g, "w").write(gtf_text)
        open(p, "w").write(psl_text)
        env = dict(os.environ, PYTHONHASHSEED="0")
        subprocess.run([sys.executable, REF, "-i", p, "-o", o, "-g", g if annotated else "None"], check=True,
                       env=env, stdout=subprocess.DEVNULL)
        return [normalise(l) for l in open(o).read().splitlines()]


def normalise(line):
    a = line.split("\t")
    return a[:6] + [sorted(a[6].split(",")) if a[6] else []]


def main():
    gtf, psl = make_input()
    out = {"gtf": gtf, "psl": psl, "annotated": run_reference(gtf, psl, True),
           "unannotated": run_reference(gtf, psl, False)}
    with open(os.path.join(HERE, "gene_vectors.json"), "w") as f:
        json.dump(out, f, indent=0)
    print(len(out["annotated"]), "lines;", sum(1 for a in out["annotated"] if a[5]), "with a best gene")


if __name__ == "__main__":
    main()
