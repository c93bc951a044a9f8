#!/usr/bin/env python3
"""Generates tests/golden/fq_vectors.json: the reference's modules F and Q (run here only).

Input (`make_input`, numpy default_rng, no reference code): a synthetic genome, isoform consensi named
like the D module's (`Isoform<k>_<reads>`), their alignments as a minimap2-style SAM, a polyA
whitelist, two read files and a reads2isoforms table.  The isoform families exercise every filter of
filterIsoforms.py: length, absolute reads, 5'/3' overhang bins (soft clips), single-exon, relative
expression, polyA extension (A-rich genome after the end, one of them whitelisted), containment by
junctions (internal ratio) and near-identical ends, on both strands and three chromosomes, plus
secondary/supplementary records, a duplicated name and small deletions that clean_psl merges.
Reference path (as Mando.py runs it): `python3 filterIsoforms.py ... --mm2_path <script that prints
the SAM> --emtrey_path emtrey.py 2> filter_reasons.txt` and `python3 assignReadsToIsoforms.py -m
<dir> -f a.fasta,b.fasta`, with a stand-in `mappy` (fastx_read and revcomp restated from mappy's
documented behaviour; mappy itself is not installed here), PYTHONHASHSEED=0, one worker.
Stored: sha256 + line counts of every output, the reason lines normalised (see `normalise`).
Nothing of the reference is copied.
"""
import hashlib
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

STUB = '''_T = {}
for _a, _b in zip("ACGTURYKMBVDHSWN", "TGCAAYRMKVBHDSWN"):
    _T[ord(_a)] = _b
    _T[ord(_a.lower())] = _b.lower()


def revcomp(s):
    return s[::-1].translate(_T)


def fastx_read(fn, read_comment=False):
    # FASTA only (the fixture's inputs): name = first word of the header
    name, seq = None, []
    for l in open(fn):
        l = l.rstrip()
        if l.startswith(">"):
            if name is not None:
                yield name, "".join(seq), None
            name, seq = l[1:].split()[0], []
        elif name is not None:
            seq.append(l.strip())
    if name is not None:
        yield name, "".join(seq), None


class Aligner:
    pass
'''

BASES = "ACGT"


def _seq(rng, n):
    return "".join(BASES[i] for i in rng.integers(0, 4, n))


def make_input(d, seed=20251016):
    """Writes genome.fa, Isoform_Consensi.fasta, iso.sam, polyAWhiteList.bed, a.fasta, b.fasta and
    reads2isoforms.txt into directory d; returns the isoform count."""
    import numpy as np

    rng = np.random.default_rng(seed)
    chroms = {"chr1": 60000, "chr2": 40000, "chrX": 30000}
    genome = {c: list(_seq(rng, n)) for c, n in chroms.items()}
    isoforms = []  # (name, chrom, strand, blocks[(s,e)], clip5, clip3, extra sam records)
    k = [0]
    polyA_white = []

    def add(chrom, strand, blocks, reads, clip5=0, clip3=0, dels=(), flag_extra=None):
        k[0] += 1
        name = f"Isoform{k[0]}_{reads}"
        isoforms.append((name, chrom, strand, blocks, clip5, clip3, dels, flag_extra))
        return name

    def arich(chrom, strand, s, e):
        # A-rich genome right after a '+' end / T-rich right before a '-' start
        g = genome[chrom]
        if strand == "+":
            for x in range(e, min(e + 15, len(g))):
                g[x] = "A" if rng.random() < 0.85 else g[x]
        else:
            for x in range(max(0, s - 15), s):
                g[x] = "T" if rng.random() < 0.85 else g[x]

    for chrom, clen in chroms.items():
        pos = 1000
        gene = 0
        while pos + 9000 < clen:
            gene += 1
            strand = "+" if rng.random() < 0.6 else "-"
            ne = int(rng.integers(3, 6))
            ex = []
            p = pos
            for i in range(ne):
                el = int(rng.integers(120, 400))
                ex.append((p, p + el))
                p += el + int(rng.integers(200, 1500))
            full = add(chrom, strand, ex, int(rng.integers(200, 900)), clip5=int(rng.integers(0, 30)),
                       clip3=int(rng.integers(0, 30)), dels=[(0, 40)] if gene % 2 else ())
            # exon skip
            if ne >= 3:
                add(chrom, strand, [ex[0]] + ex[2:], int(rng.integers(50, 200)))
            # contained in full (drop first exon, keep junctions) at low ratio -> internal filter
            add(chrom, strand, ex[1:], int(rng.integers(5, 40)))
            # near identical to full (ends within 50 nt), fewer reads -> filtered
            ex2 = [(ex[0][0] + 20, ex[0][1])] + ex[1:-1] + [(ex[-1][0], ex[-1][1] - 25)]
            add(chrom, strand, ex2, int(rng.integers(100, 190)))
            # relative expression too low
            add(chrom, strand, [ex[0], ex[-1]], 3 if rng.random() < 0.5 else 4)
            # too few reads / too short / overhang out of bins
            add(chrom, strand, ex[:2], 2)
            add(chrom, strand, [(ex[0][0], ex[0][0] + 150)], 50)
            add(chrom, strand, ex[:2] + ex[3:4] if ne > 3 else ex[:2], 60, clip5=55)
            # single exon, long enough (kept unless multi-exon-only)
            add(chrom, strand, [(ex[-1][0], ex[-1][1] + 300)], int(rng.integers(30, 80)))
            # polyA extension: a shorter 3' end with A-rich genome after it, a longer isoform covering past it
            if strand == "+":
                sh = (ex[-1][0], ex[-1][1] - 80)
                short = add(chrom, strand, ex[:-1] + [sh], int(rng.integers(60, 150)))
                arich(chrom, strand, sh[0], sh[1])
                if gene % 3 == 0:
                    polyA_white.append((chrom, sh[1] - 2, sh[1] + 2, "+"))
            else:
                sh = (ex[0][0] + 80, ex[0][1])
                short = add(chrom, strand, [sh] + ex[1:], int(rng.integers(60, 150)))
                arich(chrom, strand, sh[0], sh[1])
                if gene % 3 == 0:
                    polyA_white.append((chrom, sh[0] - 2, sh[0] + 2, "-"))
            # secondary / supplementary copies of the full isoform, and a duplicated primary name
            isoforms.append((full, chrom, strand, [(ex[0][0] + 5000, ex[0][1] + 5000)], 0, 0, (), 256))
            isoforms.append((full, chrom, strand, [(ex[1][0], ex[1][1])], 0, 0, (), 2048))
            if gene == 2:
                isoforms.append((short, chrom, strand, ex[:2], 0, 0, (), 0))
            pos = p + int(rng.integers(500, 3000))

    gseq = {c: "".join(g) for c, g in genome.items()}
    with open(os.path.join(d, "genome.fa"), "w") as fh:
        for c, s in gseq.items():
            fh.write(f">{c} synthetic\n")
            for i in range(0, len(s), 70):
                fh.write(s[i:i + 70] + "\n")
    seen = set()
    cons = []
    sam = ["@HD\tVN:1.6\tSO:unsorted"] + [f"@SQ\tSN:{c}\tLN:{n}" for c, n in chroms.items()]
    for name, chrom, strand, blocks, c5, c3, dels, extra in isoforms:
        body = "".join(gseq[chrom][s:e] for s, e in blocks)
        clip_l = c5 if strand == "+" else c3
        clip_r = c3 if strand == "+" else c5
        q = _seq(rng, clip_l) + body + _seq(rng, clip_r)
        if name not in seen and extra is None:
            seen.add(name)
            from_plus = q
            cons.append((name, from_plus if strand == "+" else from_plus[::-1].translate(str.maketrans("ACGT", "TGCA"))))
        cig = []
        if clip_l:
            cig.append(f"{clip_l}S")
        for bi, (s, e) in enumerate(blocks):
            if bi:
                cig.append(f"{s - blocks[bi - 1][1]}N")
            L = e - s
            dd = [x for x in dels if bi == 0]
            if dd and L > 80:
                a0 = dd[0][1]
                cig += [f"{a0}M", "3D", f"{L - a0 - 3}M"]
            else:
                cig.append(f"{L}M")
        if clip_r:
            cig.append(f"{clip_r}S")
        flag = (16 if strand == "-" else 0) | (extra or 0)
        nm = int(rng.integers(0, 20))
        sam.append("\t".join([name, str(flag), chrom, str(blocks[0][0] + 1), "60", "".join(cig), "*", "0", "0", q, "*",
                              f"NM:i:{nm}", "ms:i:100", "AS:i:100", "nn:i:0", "tp:A:P"]))
    with open(os.path.join(d, "Isoform_Consensi.fasta"), "w") as fh:
        for name, s in cons:
            fh.write(f">{name}\n{s}\n")
    with open(os.path.join(d, "iso.sam"), "w") as fh:
        fh.write("\n".join(sam) + "\n")
    with open(os.path.join(d, "polyAWhiteList.bed"), "w") as fh:
        for c, s, e, st in polyA_white:
            fh.write(f"{c}\t{s}\t{e}\t.\t0\t{st}\n")
    # module Q inputs: two read files, every read assigned to one isoform
    r2i = []
    for fn, tag in (("a.fasta", "A"), ("b.fasta", "B")):
        with open(os.path.join(d, fn), "w") as fh:
            for name, _ in cons:
                for j in range(int(rng.integers(1, 6))):
                    rn = f"read_{tag}_{name}_{j} extra comment"
                    fh.write(f">{rn}\n{_seq(rng, 30)}\n")
                    r2i.append(f"{rn.split()[0]}\t{name}")
    with open(os.path.join(d, "reads2isoforms.txt"), "w") as fh:
        fh.write("\n".join(r2i) + "\n")
    return len(cons)


def normalise(lines):
    """Reason texts name 'the first element' of a Python set (hash-order dependent): blank the chosen
    isoform and its read count."""
    out = []
    for l in lines:
        if "(including " in l:
            a = l.index("(including ") + len("(including ")
            l = l[:a] + "*" + l[l.index(")", a):]
        if "contained in) " in l and " and expressed at " in l:
            a = l.index("contained in) ") + len("contained in) ")
            l = l[:a] + "*" + l[l.index(" and expressed at ", a):]
            a = l.index(" reads compared to ") + len(" reads compared to ")
            l = l[:a] + "*" + l[l.index(" reads for the isoform", a):]
        if "almost identical to " in l:
            l = l[:l.index("almost identical to ") + len("almost identical to ")] + "*"
        out.append(l)
    return out


def _digest(path):
    data = open(path, "rb").read()
    return {"lines": data.count(b"\n"), "sha256": hashlib.sha256(data).hexdigest()}


REF_ARGS = ["-r", "0.01", "-R", "3", "-O", "0,40,0,40", "-t", "1", "-A", "0.5", "-s", "1", "-d", "50",
            "-I", "200"]


def main():
    out = {"input": "tests/golden/make_fq_vectors.py make_input()", "args": REF_ARGS}
    with tempfile.TemporaryDirectory(dir="/tmp") as tmp:
        stub = os.path.join(tmp, "stub", "mappy")
        os.makedirs(stub)
        open(os.path.join(stub, "__init__.py"), "w").write(STUB)
        env = dict(os.environ, PYTHONPATH=os.path.join(tmp, "stub"), PYTHONHASHSEED="0")
        for multi, nratio in ((0, "1"), (1, "0.1")):
            d = os.path.join(tmp, f"m{multi}")
            os.makedirs(d)
            out["isoforms"] = make_input(d)
            mm2 = os.path.join(d, "fake_mm2.sh")
            with open(mm2, "w") as fh:
                fh.write(f"#!/bin/sh\ncat {os.path.join(d, 'iso.sam')}\n")
            os.chmod(mm2, 0o755)
            with open(os.path.join(d, "filter_reasons.txt"), "w") as err:
                subprocess.run([sys.executable, "/root/reference/filterIsoforms.py", "-p", d, "-i",
                                os.path.join(d, "Isoform_Consensi.fasta"), "-G", os.path.join(d, "genome.fa"),
                                "-m", "/root/reference", "-M", str(multi), "-n", nratio, "--mm2_path", mm2,
                                "--emtrey_path", "/root/reference/emtrey.py"] + REF_ARGS,
                               check=True, env=env, stderr=err, stdout=subprocess.DEVNULL, cwd=d)
            r = {"internal_ratio": float(nratio)}
            for f in ("Isoforms.filtered.fasta", "Isoforms.filtered.clean.psl", "Isoforms.filtered.clean.gtf",
                      "Isoforms.aligned.out.clean.psl"):
                r[f] = _digest(os.path.join(d, f))
            r["reasons"] = normalise(open(os.path.join(d, "filter_reasons.txt")).read().split("\n")[:-1])
            if multi == 0:
                subprocess.run([sys.executable, "/root/reference/assignReadsToIsoforms.py", "-m", d, "-f",
                                f"{os.path.join(d, 'a.fasta')},{os.path.join(d, 'b.fasta')}"],
                               check=True, env=env, stdout=subprocess.DEVNULL, cwd=d)
                for f in ("Isoforms.filtered.clean.quant", "Isoforms.filtered.clean.tpm"):
                    data = open(os.path.join(d, f)).read()
                    # the header names the read files by path: store it relative
                    r[f] = {"sha256_body": hashlib.sha256("\n".join(data.split("\n")[1:]).encode()).hexdigest(),
                            "lines": data.count("\n")}
            out[f"multi{multi}"] = r
    dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fq_vectors.json")
    json.dump(out, open(dst, "w"), indent=1)
    print("wrote", dst, {k: {f: v["lines"] for f, v in r.items() if isinstance(v, dict) and "lines" in v}
                         for k, r in out.items() if k.startswith("multi")})


if __name__ == "__main__":
    main()
