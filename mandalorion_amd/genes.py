"""Gene grouping of the filtered isoforms (groupIsoforms.py, run by Mando.py:458-469 after module F).

Host-side row beyond the D module.  The reference marks every second base of every annotated exon in
a per-base dict of gene sets (groupIsoforms.py:28-83) and then counts, per isoform locus, the covered
bases that carry each gene (groupIsoforms.py:142-171).  Here the same counts come from interval
arithmetic, without per-base tables:

- An exon [s, e) marks s, s+2, ... < e, i.e. the positions of s's parity inside [s, e).  So a gene's
  marked set is (even positions of the union of its even-start exons) ∪ (odd positions of the union
  of its odd-start exons), for the chromosome of its first exon line (groupIsoforms.py:59-60, :72).
- A locus covers the union of its isoforms' blocks (groupIsoforms.py:145-153); the count of a gene is
  the number of even (odd) covered positions inside its even (odd) union.

Output lines and their order follow groupIsoforms.py:84-186 (strand '+' then '-', isoforms in file
order, a new locus when the chromosome changes or an isoform starts after the running locus end,
locus numbers restarting per strand; best gene = max (count, name)).  The one difference: the
reference joins the overlapping genes in Python set order, which depends on the hash seed; here they
are joined in sorted order.
"""
from __future__ import annotations

import gzip

import numpy as np


def _merge(iv: list[tuple[int, int]]) -> tuple[np.ndarray, np.ndarray]:
    iv = sorted(x for x in iv if x[1] > x[0])
    s, e = [], []
    for a, b in iv:
        if s and a <= e[-1]:
            e[-1] = max(e[-1], b)
        else:
            s.append(a)
            e.append(b)
    return np.asarray(s, dtype=np.int64), np.asarray(e, dtype=np.int64)


def _count_parity(cs, ce, gs, ge, odd: bool) -> int:
    """Positions of one parity in (∪[cs,ce)) ∩ (∪[gs,ge)); both lists merged and sorted."""
    if len(gs) == 0 or len(cs) == 0:
        return 0
    # every pair of overlapping intervals (both lists are disjoint and sorted)
    i = np.searchsorted(ge, cs, side="right")          # first gene interval ending after cs
    j = np.searchsorted(gs, ce, side="left")           # first gene interval starting at/after ce
    tot = 0
    for k in np.nonzero(j > i)[0]:
        a = np.maximum(gs[i[k]:j[k]], cs[k])
        b = np.minimum(ge[i[k]:j[k]], ce[k])
        if odd:
            tot += int((b // 2 - a // 2).sum())
        else:
            tot += int(((b + 1) // 2 - (a + 1) // 2).sum())
    return tot


class Annotation:
    """read_annotation (groupIsoforms.py:28-83) as per-(strand, chromosome) gene interval tables."""

    def __init__(self, gtf: str):
        genes: dict[str, dict[str, list]] = {"+": {}, "-": {}}
        if gtf != "None":
            if gtf.endswith(".gtf.gz"):
                f = gzip.open(gtf, "rt")
            elif gtf.endswith(".gtf"):
                f = open(gtf)
            else:
                raise ValueError(f"{gtf}: annotation must end in .gtf or .gtf.gz (groupIsoforms.py:40-43)")
            with f:
                for line in f:
                    if line[0] == "#":
                        continue
                    a = line.strip().split("\t")
                    name = a[8].split('gene_id "')[1].split('"')[0]
                    if a[2] != "exon":
                        continue
                    if "gene_name" in a[8]:
                        name += "_" + a[8].split('gene_name "')[1].split('"')[0]
                    g = genes[a[6]].setdefault(name, [a[0], []])
                    g[1].append((int(a[3]) - 1, int(a[4])))
        # (strand, chrom) -> (names, span starts, span ends, [(even union), (odd union)])
        self.tables: dict[tuple[str, str], tuple] = {}
        for strand in "+-":
            per: dict[str, list] = {}
            for name, (chrom, exons) in genes[strand].items():
                ev = _merge([x for x in exons if x[0] % 2 == 0])
                od = _merge([x for x in exons if x[0] % 2 == 1])
                lo = min(x[0] for x in exons)
                hi = max(x[1] for x in exons)
                per.setdefault(chrom, []).append((name, lo, hi, ev, od))
            for chrom, rows in per.items():
                self.tables[(strand, chrom)] = (
                    [r[0] for r in rows], np.asarray([r[1] for r in rows], dtype=np.int64),
                    np.asarray([r[2] for r in rows], dtype=np.int64), [(r[3], r[4]) for r in rows])

    def match(self, strand: str, chrom: str, blocks: list[tuple[int, int]]) -> tuple[str, str]:
        """match_isoforms (groupIsoforms.py:142-186): (best gene, overlapping genes)."""
        t = self.tables.get((strand, chrom))
        if t is None or not blocks:
            return "", ""
        cs, ce = _merge(blocks)
        if len(cs) == 0:
            return "", ""
        names, lo, hi, unions = t
        counts = []
        for k in np.nonzero((lo < ce[-1]) & (hi > cs[0]))[0]:
            (es, ee), (os_, oe) = unions[k]
            n = _count_parity(cs, ce, es, ee, False) + _count_parity(cs, ce, os_, oe, True)
            if n:
                counts.append((n, names[k]))
        if not counts:
            return "", ""
        return max(counts)[1], ",".join(sorted(c[1] for c in counts))


def group_isoforms(sorted_psl: str, out_file: str, genome_annotation: str = "None") -> int:
    """groupIsoforms.py -i sorted_psl -o out_file -g genome_annotation; returns loci written."""
    ann = Annotation(genome_annotation)
    with open(sorted_psl) as f:
        rows = [ln.strip().split("\t") for ln in f]
    nloci = 0
    with open(out_file, "w") as out:
        for strand in "+-":
            locus = 0
            group: list[list[str]] = []
            chrom, start, end = "", 0, 0

            def flush():
                nonlocal locus
                blocks = []
                for a in group:
                    ts = a[20].split(",")[:-1]
                    ws = a[18].split(",")[:-1]
                    blocks += [(int(s), int(s) + int(w)) for s, w in zip(ts, ws)]
                best, overl = ann.match(strand, chrom, blocks)
                locus += 1
                for a in group:
                    out.write(f"{a[9]}\tLocus{locus}\t{chrom}\t{start}\t{end}\t{best}\t{overl}\n")

            for a in rows:
                if a[8] != strand:
                    continue
                c, s, e = a[13], int(a[15]), int(a[16])
                if c == chrom and s <= end:
                    end = max(end, e)
                    group.append(a)
                    continue
                if group:
                    flush()
                group, chrom, start, end = [a], c, s, e
            if group:
                flush()
            nloci += locus
    return nloci
