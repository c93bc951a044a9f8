"""Synthetic module F inputs for the host / device comparisons (tests/test_modf_gpu.py): a genome, the
consensi FASTA, a clean PSL of isoforms built from shared exon sets per locus (so that containment,
near-identical ends, polyA extension and the whitelist all fire), and a polyA whitelist BED."""
import os
import random

import numpy as np


def write_inputs(d, n_loci=300, seed=3, chroms=3):
    rng = random.Random(seed)
    nrg = np.random.default_rng(seed)
    genome = {}
    per = n_loci // chroms
    for c in range(chroms):
        seq = np.frombuffer(b"ACGT", dtype=np.uint8)[nrg.integers(0, 4, size=per * 4000 + 20000)].copy()
        # A-rich (and T-rich) stretches, some at exon ends, for the polyA extension test
        for p in nrg.integers(100, len(seq) - 100, size=max(1, per // 2)):
            base = b"AAAAT" if nrg.random() < 0.5 else b"TTTTA"
            seq[p:p + 20] = np.frombuffer(base, dtype=np.uint8)[nrg.integers(0, 5, size=20)]
        genome[f"chr{c + 1}"] = seq.tobytes().decode()
    with open(os.path.join(d, "genome.fa"), "w") as fh:
        for name, seq in genome.items():
            fh.write(f">{name}\n")
            fh.write("\n".join(seq[k:k + 80] for k in range(0, len(seq), 80)) + "\n")
    lines, cons, wl = [], [], []
    iso_id = 0
    for c in range(chroms):
        chrom = f"chr{c + 1}"
        for loc in range(per):
            base = 5000 + loc * 4000
            nex = rng.randrange(1, 6)
            exons, p = [], base
            for _ in range(nex):
                ln = rng.randrange(120, 520)
                exons.append((p, p + ln))
                p += ln + rng.randrange(80, 600)
            strand = rng.choice("+-")
            for v in range(rng.randrange(1, 7)):
                # a variant: a sub-range of the exons, ends jittered, sometimes a shifted junction
                a = rng.randrange(0, nex)
                b = rng.randrange(a, nex)
                ex = [list(e) for e in exons[a:b + 1]]
                ex[0][0] += rng.choice([0, 0, 3, -4, 25, 60])
                ex[-1][1] += rng.choice([0, 0, -2, 5, -30, 40])
                if len(ex) > 1 and rng.random() < 0.15:
                    ex[0][1] += rng.choice([-2, 2, 7])
                if any(e[1] <= e[0] for e in ex):
                    continue
                ab = rng.choice([0, 1, 2, 3, 5, 8, 13, 40, 100]) if rng.random() < 0.03 else rng.randrange(1, 120)
                name = f"Isoform{iso_id}_{ab}"
                iso_id += 1
                sizes = [e[1] - e[0] for e in ex]
                qsize = sum(sizes)
                qs, qe = rng.choice([(0, qsize), (0, qsize), (2, qsize), (0, qsize - 3), (40, qsize)])
                if qe <= qs:
                    continue
                qstarts, q = [], 0
                for sz in sizes:
                    qstarts.append(q)
                    q += sz
                f = [str(qsize), "0", "0", "0", "0", "0", "0", "0", strand, name, str(qsize), str(qs), str(qe), chrom,
                     str(len(genome[chrom])), str(ex[0][0]), str(ex[-1][1]), str(len(ex)),
                     ",".join(map(str, sizes)) + ",", ",".join(map(str, qstarts)) + ",",
                     ",".join(str(e[0]) for e in ex) + ","]
                lines.append("\t".join(f))
                cons.append((name, "".join(rng.choice("ACGT") for _ in range(min(qsize, 200)))))
                if rng.random() < 0.2:
                    pos = ex[-1][1] if strand == "+" else ex[0][0]
                    wl.append(f"{chrom}\t{pos - 2}\t{pos + 3}\tx\t0\t{strand}")
    rng.shuffle(lines)
    with open(os.path.join(d, "clean.psl"), "w") as fh:
        fh.write("\n".join(lines) + "\n")
    with open(os.path.join(d, "Isoform_Consensi.fasta"), "w") as fh:
        for name, s in cons:
            fh.write(f">{name}\n{s}\n")
    with open(os.path.join(d, "polyAWhiteList.bed"), "w") as fh:
        fh.write("\n".join(wl) + "\n")
    return len(lines)
