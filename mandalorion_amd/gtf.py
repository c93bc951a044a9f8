"""Annotated splice sites and poly(A) white list from a GTF (host side, cold path).

Restates `parse_genome` (/root/reference/utils/SpliceDefineConsensus.py:334-389) and the per-locus
bound filter of defineIsoforms.main (/root/reference/defineIsoforms.py:135-150), including its string
(not numeric) comparisons of exon starts/ends against the transcript start/end.
"""
from __future__ import annotations

import gzip


def parse_genome(path: str, white_list_polyA: list[str]):
    """Returns (chrom_list, left_bounds, right_bounds, polyAWhiteList) like the reference."""
    poly = []
    chroms = set()
    genes: dict[str, list] = {}
    left: dict[str, dict] = {}
    right: dict[str, dict] = {}
    fh = gzip.open(path, "rt") if path.endswith(".gtf.gz") else open(path)
    with fh:
        for line in fh:
            pawl = any(el in line for el in white_list_polyA)
            a = line.strip().split("\t")
            if len(a) <= 7:
                continue
            if a[2] == "exon":
                key = a[8].split('transcript_id "')[1].split('"')[0]
                genes.setdefault(key, []).append((a[0], a[3], a[4], a[6], pawl))
    for tid, data in genes.items():
        chrom = data[0][0]
        chroms.add(chrom)
        if chrom not in right:
            left[chrom] = {"5": [], "3": []}
            right[chrom] = {"5": [], "3": []}
        start = sorted(data, key=lambda x: int(x[1]))[0][1]
        end = sorted(data, key=lambda x: int(x[2]), reverse=True)[0][2]
        direction = data[0][3]
        if data[0][4]:
            if direction == "+":
                poly.append((chrom, direction, end, tid))
            elif direction == "-":
                poly.append((chrom, direction, start, tid))
        for e in data:
            if e[1] != start:
                if e[3] == "+":
                    right[chrom]["3"].append(int(e[1]) - 1)
                elif e[3] == "-":
                    right[chrom]["5"].append(int(e[1]) - 1)
            if e[2] != end:
                if e[3] == "+":
                    left[chrom]["5"].append(int(e[2]))
                if e[3] == "-":
                    left[chrom]["3"].append(int(e[2]))
    return chroms, left, right, poly


def locus_bounds(left: dict, right: dict, chrom: str, start: int, end: int) -> list[list[int]]:
    """[left '5', left '3', right '5', right '3'] annotated positions with start < pos < end."""
    lb = left.get(chrom, {"5": [], "3": []})
    rb = right.get(chrom, {"5": [], "3": []})
    return [[p for p in lb["5"] if start < p < end], [p for p in lb["3"] if start < p < end],
            [p for p in rb["5"] if start < p < end], [p for p in rb["3"] if start < p < end]]


class BoundsIndex:
    """locus_bounds for many loci: each chromosome's four position lists sorted once, every locus a
    pair of binary searches (the lists' order does not matter downstream: make_genome_bins sorts them,
    SDC:396-399).  Equal to [sorted(x) for x in locus_bounds(...)]."""

    def __init__(self, left: dict, right: dict):
        import numpy as np

        self.np = np
        self.idx = {}
        for chrom in set(left) | set(right):
            lb = left.get(chrom, {"5": [], "3": []})
            rb = right.get(chrom, {"5": [], "3": []})
            self.idx[chrom] = [np.sort(np.asarray(x, dtype=np.int64)) for x in (lb["5"], lb["3"], rb["5"], rb["3"])]

    def __bool__(self):
        return bool(self.idx)

    def bounds(self, chrom: str, start: int, end: int):
        np = self.np
        lists = self.idx.get(chrom)
        if lists is None:
            return [np.zeros(0, np.int64)] * 4
        return [a[np.searchsorted(a, start, "right"):np.searchsorted(a, end, "left")] for a in lists]


def write_polya_bed(path: str, poly: list, white_list_polyA: list[str]) -> None:
    """polyAWhiteList.bed exactly as defineIsoforms.main writes it (:111-120)."""
    with open(path, "w") as out:
        if "0" not in white_list_polyA:
            for chrom, direction, end, tid in poly:
                p = int(end)
                out.write("%s\t%s\t%s\t%s\t%s\t%s\n" % (chrom, str(p - 20), str(p + 20), tid, "0", direction))
