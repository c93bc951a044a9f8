"""Synthetic D-module inputs: spliced loci written as Mandalorion locus PSL files (tmp_SS/*.psl).

There is no network and no SIRV / gencode data in the image, so every D-module test and benchmark runs
on loci made here (SURVEY.md §8d "Synthetic inputs"):
  * per locus a random genome segment with 1..N exons, GT..AG introns (5 % GC..AG);
  * 1..3 isoforms by skipping one internal exon; TSS/TES jitter of +-3 nt;
  * reads are noisy copies of an isoform (R2C2 model: 1 % substitutions, 0.5 % insertions, 0.5 %
    deletions, indels twice as likely in homopolymers), aligned back to the genome exactly as the
    generator made them, giving the 24-column "Mando PSL" of SURVEY.md Appendix A with a
    minimap2 `--cs=long` string (`=ACGT`, `*ag`, `+acg`, `-acg`, `~gt500ag`) and the read sequence.
Blocks are whole exons, i.e. what `clean_psl` (reference SpliceDefineConsensus.py:14-92) leaves after
merging gaps < 10 nt.  Loci are written one file per locus named `chrom~start~end.psl` with start/end
the min tStart / max tEnd of the locus' reads, lines in (tStart, tEnd) order, exactly the layout that
`get_chromosomes` (SpliceDefineConsensus.py:442-495) produces from the sorted clean PSL.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field

import numpy as np

DATA_SEED = 20250117
_B = np.frombuffer(b"ACGT", dtype=np.uint8)
R2C2 = dict(sub=0.010, ins=0.005, dele=0.005)
PACBIO = dict(sub=0.0005, ins=0.00025, dele=0.00025)


@dataclass
class LocusSpec:
    n_reads: int = 5
    exons: tuple[int, int] = (4, 8)          # exon count range (1 => mono-exon locus)
    exon_len: tuple[int, int] = (100, 300)
    intron_len: tuple[int, int] = (300, 3000)
    isoforms: tuple[int, int] = (1, 3)
    model: dict = field(default_factory=lambda: dict(R2C2))
    jitter: int = 3
    annotate: bool = False                   # also emit GTF transcripts for this locus


@dataclass
class Locus:
    chrom: str
    start: int
    end: int
    lines: list[str]
    gtf: list[str]
    isoform_of_read: list[int]

    @property
    def root(self) -> str:
        return f"{self.chrom}~{self.start}~{self.end}"


def _rand_seq(rng, n):
    return _B[rng.integers(0, 4, size=n)].tobytes().decode()


def _hp_mask(t: str) -> np.ndarray:
    a = np.frombuffer(t.encode(), dtype=np.uint8)
    hp = np.zeros(len(a), dtype=bool)
    if len(a) > 1:
        same = a[1:] == a[:-1]
        hp[1:] |= same
        hp[:-1] |= same
    return hp


def _align_exon(rng, ref: str, model: dict, first: bool, last: bool):
    """Noisy copy of one exon segment; returns (query, cs ops list of (op, text), counts)."""
    n = len(ref)
    f = np.where(_hp_mask(ref), 2.0, 1.0)
    u = rng.random(n)
    ins_u = rng.random(n)
    ins_pick = rng.random(n)
    ins_base = rng.integers(0, 4, size=n)
    sub_shift = rng.integers(1, 4, size=n)
    ops: list[list] = []
    q = []
    cnt = dict(match=0, mis=0, qins=0, qbase=0, tins=0, tbase=0)

    def push(op, text):
        if ops and ops[-1][0] == op and op in "=+-":
            ops[-1][1] += text
        else:
            ops.append([op, text])

    for i, c in enumerate(ref):
        edge = (first and i == 0) or (last and i == n - 1)
        pd = model["dele"] * f[i]
        if not edge and u[i] < pd:
            push("-", c.lower())
            cnt["tbase"] += 1
        elif not edge and u[i] < pd + model["sub"]:
            qb = "ACGT"[("ACGT".index(c) + int(sub_shift[i])) % 4]
            push("*", c.lower() + qb.lower())
            q.append(qb)
            cnt["mis"] += 1
        else:
            push("=", c)
            q.append(c)
            cnt["match"] += 1
        if not (last and i == n - 1) and ins_u[i] < model["ins"] * f[i]:
            b = c if ins_pick[i] < 0.5 else "ACGT"[int(ins_base[i])]
            push("+", b.lower())
            q.append(b)
            cnt["qbase"] += 1
    cnt["qins"] = sum(1 for o in ops if o[0] == "+")
    cnt["tins"] = sum(1 for o in ops if o[0] == "-")
    return "".join(q), ops, cnt


def make_locus(rng, chrom: str, g0: int, spec: LocusSpec, name_prefix: str) -> tuple[Locus, int]:
    """One locus starting at genome position g0; returns (locus, genome end used)."""
    n_ex = int(rng.integers(spec.exons[0], spec.exons[1] + 1))
    ex_len = rng.integers(spec.exon_len[0], spec.exon_len[1] + 1, size=n_ex)
    in_len = rng.integers(spec.intron_len[0], spec.intron_len[1] + 1, size=max(n_ex - 1, 0))
    pad = 50
    total = int(ex_len.sum() + in_len.sum()) + 2 * pad
    g = list(_rand_seq(rng, total))
    exons = []  # (genome start, genome end) absolute, half-open
    p = pad
    for k in range(n_ex):
        exons.append((g0 + p, g0 + p + int(ex_len[k])))
        p += int(ex_len[k])
        if k < n_ex - 1:
            il = int(in_len[k])
            donor = "GC" if rng.random() < 0.05 else "GT"
            g[p:p + 2] = list(donor)
            g[p + il - 2:p + il] = list("AG")
            p += il
    genome = "".join(g)

    def gseq(a, b):
        return genome[a - g0:b - g0]

    # isoforms: full, plus skips of distinct internal exons
    n_iso = int(rng.integers(spec.isoforms[0], spec.isoforms[1] + 1))
    isoforms = [list(range(n_ex))]
    internal = list(range(1, n_ex - 1))
    rng.shuffle(internal)
    for k in internal[:max(0, n_iso - 1)]:
        isoforms.append([e for e in range(n_ex) if e != k])
    lines_keyed = []
    iso_of = []
    for r in range(spec.n_reads):
        iso = int(rng.integers(0, len(isoforms)))
        ex = [exons[e] for e in isoforms[iso]]
        js = int(rng.integers(-spec.jitter, spec.jitter + 1))
        je = int(rng.integers(-spec.jitter, spec.jitter + 1))
        ex[0] = (ex[0][0] + js, ex[0][1])
        ex[-1] = (ex[-1][0], ex[-1][1] + je)
        qparts, cs = [], []
        tot = dict(match=0, mis=0, qins=0, qbase=0, tins=0, tbase=0)
        for k, (a, b) in enumerate(ex):
            qseg, ops, cnt = _align_exon(rng, gseq(a, b), spec.model, k == 0, k == len(ex) - 1)
            qparts.append(qseg)
            cs.extend(op + txt for op, txt in ops)
            for key in tot:
                tot[key] += cnt[key]
            if k < len(ex) - 1:
                na = ex[k + 1][0]
                il = na - b
                cs.append("~" + gseq(b, b + 2).lower() + str(il) + gseq(na - 2, na).lower())
        query = "".join(qparts)
        bsizes = [b - a for a, b in ex]
        tstarts = [a for a, _ in ex]
        qstarts, qq = [], 0
        for s in bsizes:
            qstarts.append(qq)
            qq += s
        introns = sum(ex[k + 1][0] - ex[k][1] for k in range(len(ex) - 1))
        alen = tot["match"] + tot["mis"] + tot["qbase"] + tot["tbase"]
        acc = tot["match"] / alen if alen else 1.0
        name = f"{name_prefix}r{r}"
        cols = [tot["match"], tot["mis"], 0, introns, tot["qins"], tot["qbase"], tot["tins"], tot["tbase"],
                "+", name, len(query), 0, len(query), chrom, 250_000_000, ex[0][0], ex[-1][1], len(ex),
                ",".join(map(str, bsizes)) + ",", ",".join(map(str, qstarts)) + ",",
                ",".join(map(str, tstarts)) + ",", f"{acc:.4f}", "".join(cs), query]
        line = "\t".join(str(c) for c in cols)
        lines_keyed.append((ex[0][0], ex[-1][1], line, iso))
    lines_keyed.sort(key=lambda t: (t[0], t[1], t[2]))
    lines = [t[2] for t in lines_keyed]
    iso_of = [t[3] for t in lines_keyed]
    start = min(t[0] for t in lines_keyed)
    end = max(t[1] for t in lines_keyed)
    gtf = []
    if spec.annotate:
        for i, iso in enumerate(isoforms):
            tid = f"{name_prefix}T{i}"
            for e in iso:
                a, b = exons[e]
                gtf.append(f'{chrom}\tsim\texon\t{a + 1}\t{b}\t.\t+\t.\tgene_id "{name_prefix}G"; '
                           f'transcript_id "{tid}"; tag "basic";')
    return Locus(chrom, start, end, lines, gtf, iso_of), g0 + total


def make_dataset(specs: list[LocusSpec], seed: int = DATA_SEED, chroms: int = 2, gap: int = 5000) -> list[Locus]:
    """Loci for the given specs, spread round-robin over `chroms` chromosomes, non-overlapping."""
    rng = np.random.default_rng(seed)
    pos = {f"chr{c + 1}": 10_000 for c in range(chroms)}
    out = []
    for i, sp in enumerate(specs):
        chrom = f"chr{i % chroms + 1}"
        loc, gend = make_locus(rng, chrom, pos[chrom], sp, f"L{i}_")
        pos[chrom] = gend + gap
        out.append(loc)
    return out


def write_dataset(loci: list[Locus], path: str, gtf_name: str = "annotation.gtf") -> dict:
    """Writes <path>/tmp_SS/<root>.psl per locus (+ annotation.gtf if any locus is annotated)."""
    ss = os.path.join(path, "tmp_SS")
    os.makedirs(ss, exist_ok=True)
    n = 0
    for loc in loci:
        with open(os.path.join(ss, loc.root + ".psl"), "w") as fh:
            for ln in loc.lines:
                fh.write(ln + "\n")
                n += 1
    gtf = [g for loc in loci for g in loc.gtf]
    gtf_path = None
    if gtf:
        gtf_path = os.path.join(path, gtf_name)
        with open(gtf_path, "w") as fh:
            fh.write("\n".join(gtf) + "\n")
    return {"records": n, "loci": len(loci), "gtf": gtf_path}


def fixture_specs() -> list[LocusSpec]:
    """The loci behind tests/golden/cluster_vectors.json: config-1-shaped (5 reads x ~1 kb) plus
    deeper, mono-exon, annotated and low-count cases."""
    sp = []
    for k in range(10):
        sp.append(LocusSpec(n_reads=5, exons=(3, 6), exon_len=(120, 300), intron_len=(300, 1500)))
    for k in range(4):
        sp.append(LocusSpec(n_reads=30, exons=(4, 8), exon_len=(100, 400), intron_len=(300, 2000),
                            isoforms=(2, 3)))
    for k in range(3):
        sp.append(LocusSpec(n_reads=8, exons=(1, 1), exon_len=(600, 1200)))
    for k in range(3):
        sp.append(LocusSpec(n_reads=12, exons=(4, 7), exon_len=(100, 300), intron_len=(300, 1500),
                            annotate=True))
    sp.append(LocusSpec(n_reads=2, exons=(3, 4), exon_len=(100, 200)))
    sp.append(LocusSpec(n_reads=60, exons=(5, 9), exon_len=(80, 250), intron_len=(300, 3000),
                        isoforms=(3, 3)))
    sp.append(LocusSpec(n_reads=150, exons=(4, 6), exon_len=(100, 250), intron_len=(300, 1200),
                        isoforms=(3, 3)))
    sp.append(LocusSpec(n_reads=20, exons=(4, 6), exon_len=(100, 250), intron_len=(300, 1200),
                        model=dict(sub=0.04, ins=0.03, dele=0.03)))
    sp.append(LocusSpec(n_reads=520, exons=(3, 4), exon_len=(80, 200), intron_len=(300, 800),
                        isoforms=(1, 2)))
    return sp
