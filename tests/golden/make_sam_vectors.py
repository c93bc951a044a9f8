#!/usr/bin/env python3
"""Generates tests/golden/sam_vectors.json: the reference's SAM -> PSL -> clean PSL (run here only).

Input (`make_input`, numpy default_rng, no reference code): a synthetic minimap2-style SAM — @SQ
header lines, mapped records on three chromosomes with CIGARs mixing M / I / D / N / S / H / = / X,
flags 0 / 16 / 256 / 272 / 2048, unmapped records (RNAME '*'), NM / nn / ts / tp / cs:Z tags in
varying order and presence (no cs tag only in the non-mando pass), read sequences with IUPAC bytes,
and reads with several records (clean_psl's primary filter).
Reference path: `python3 /root/reference/emtrey.py -i in.sam -o out.psl [-m] -t 2 -b 37`
(Mando.py:336-341; the small batch exercises emtrey's batch boundaries) and the reference's clean_psl
(SpliceDefineConsensus.py:14-92, primary=True and False), with a stand-in `mappy` module whose
`revcomp` restates mappy's (minimap2 seq_comp_table, IUPAC complements either case, other bytes kept,
as in mandalorion_amd/csrc/revcomp.h) — mappy itself is not installed here.
Stored: line counts, per-line sha256 prefixes and whole-file sha256 of every output.  Nothing of the
reference is copied.
"""
import hashlib
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

BASES = "ACGT"
IUPAC = "ACGTNRYKMacgtn"


def _seq(rng, n, iupac=False):
    alpha = IUPAC if iupac else BASES
    return "".join(alpha[i] for i in rng.integers(0, len(alpha), n))


def _cs(rng, ops):
    """A cs:Z long-form string shaped like the CIGAR (its content is carried through, not checked)."""
    out = []
    for n, op in ops:
        if op in "M=X":
            k = 0
            while k < n:
                run = int(min(n - k, rng.integers(1, 60)))
                if rng.random() < 0.2 and run == 1:
                    out.append("*" + _seq(rng, 1).lower() + _seq(rng, 1).lower())
                else:
                    out.append("=" + _seq(rng, run))
                k += run
        elif op == "I":
            out.append("+" + _seq(rng, n).lower())
        elif op == "D":
            out.append("-" + _seq(rng, n).lower())
        elif op == "N":
            out.append("~gt" + str(n) + "ag")
    return "".join(out)


def make_input(path, n_reads=160, seed=20251015, with_cs=True):
    import numpy as np

    rng = np.random.default_rng(seed)
    chroms = [("chr1", 248956422), ("chr2", 242193529), ("chrM", 16569)]
    lines = ["@HD\tVN:1.6\tSO:unsorted"] + [f"@SQ\tSN:{c}\tLN:{n}" for c, n in chroms]
    n_rec = 0
    for r in range(n_reads):
        name = f"read_{r}_{int(rng.integers(0, 10**6))}"
        n_hits = 1 if rng.random() < 0.8 else int(rng.integers(2, 4))
        for h in range(n_hits):
            if rng.random() < 0.06:
                lines.append(f"{name}\t4\t*\t0\t0\t*\t*\t0\t0\t{_seq(rng, 50)}\t*")
                continue
            ops = []
            if rng.random() < 0.5:
                ops.append((int(rng.integers(1, 40)), "S" if rng.random() < 0.8 else "H"))
            n_blocks = int(rng.integers(1, 7))
            use_eqx = rng.random() < 0.1
            for b in range(n_blocks):
                m = int(rng.integers(15, 300))
                if use_eqx:
                    x = int(rng.integers(0, 3))
                    # keep an M so that emtrey's accuracy denominator (M + I + D + nn) is never 0
                    ops += [(m, "="), (1, "X"), (3, "M")] if x else [(m, "="), (2, "M")]
                else:
                    ops.append((m, "M"))
                if b + 1 < n_blocks:
                    u = rng.random()
                    if u < 0.25:
                        ops.append((int(rng.integers(1, 6)), "I"))
                        ops.append((int(rng.integers(10, 60)), "M"))
                    if u < 0.45:
                        ops.append((int(rng.integers(1, 12)), "D"))
                    elif u < 0.55:
                        ops.append((int(rng.integers(2, 10)), "N"))  # short intron: merged by clean_psl
                    else:
                        ops.append((int(rng.integers(40, 20000)), "N"))
            if rng.random() < 0.5:
                ops.append((int(rng.integers(1, 40)), "S" if rng.random() < 0.8 else "H"))
            qlen = sum(n for n, op in ops if op in "MIS=X")
            chrom, clen = chroms[int(rng.integers(0, 3 if rng.random() < 0.05 else 2))]
            pos = int(rng.integers(1, max(2, clen - 10**6)))
            flag = [0, 16][int(rng.integers(0, 2))] if h == 0 else [256, 272, 2048, 2064][int(rng.integers(0, 4))]
            n_m = sum(n for n, op in ops if op == "M")
            id_ = sum(n for n, op in ops if op in "ID")
            tags = []
            nm = id_ + int(rng.integers(-3, 12))  # may undercut I+D: emtrey clamps the mismatch count at 0
            if rng.random() < 0.95:
                tags.append(f"NM:i:{max(0, nm)}")
            tags += [f"ms:i:{int(rng.integers(0, 3000))}", f"AS:i:{int(rng.integers(0, 3000))}"]
            if rng.random() < 0.7:
                tags.append(f"nn:i:{int(rng.integers(0, 3)) if rng.random() < 0.3 else 0}")
            if rng.random() < 0.8:
                tags.append("tp:A:" + ("P" if h == 0 else "S"))
            if rng.random() < 0.75:
                tags.append("ts:A:" + ("+" if rng.random() < 0.5 else "-"))
            if with_cs:
                tags.append("cs:Z:" + _cs(rng, ops))
            order = rng.permutation(len(tags))
            tags = [tags[i] for i in order]
            seq = _seq(rng, qlen, iupac=rng.random() < 0.3)
            cigar = "".join(f"{n}{op}" for n, op in ops)
            mapq = int(rng.integers(0, 61))
            lines.append("\t".join([name, str(flag), chrom, str(pos), str(mapq), cigar, "*", "0", "0", seq, "*"] + tags))
            n_rec += 1
    with open(path, "w") as fh:
        fh.write("\n".join(lines) + "\n")
    return n_rec


def _digest(path):
    data = open(path, "rb").read()
    lines = data.split(b"\n")[:-1]
    return {"lines": len(lines), "sha256": hashlib.sha256(data).hexdigest(),
            "line_sha": [hashlib.sha256(l).hexdigest()[:16] for l in lines]}


STUB = '''_T = {}
for _a, _b in zip("ACGTURYKMBVDHSWN", "TGCAAYRMKVBHDSWN"):
    _T[ord(_a)] = _b
    _T[ord(_a.lower())] = _b.lower()


def revcomp(s):
    return s[::-1].translate(_T)


class Aligner:
    pass
'''


def main():
    out = {"input": "tests/golden/make_sam_vectors.py make_input()"}
    with tempfile.TemporaryDirectory(dir="/tmp") as tmp:
        stub = os.path.join(tmp, "stub", "mappy")
        os.makedirs(stub)
        open(os.path.join(stub, "__init__.py"), "w").write(STUB)
        env = dict(os.environ, PYTHONPATH=os.path.join(tmp, "stub"))
        sys.path.insert(0, os.path.join(tmp, "stub"))
        sys.path.insert(0, "/root/reference/utils")
        import SpliceDefineConsensus as S

        for tag, with_cs, mflag in (("mando", True, ["-m"]), ("plain", False, [])):
            sam = os.path.join(tmp, f"{tag}.sam")
            out[tag + "_records"] = make_input(sam, with_cs=with_cs)
            psl = os.path.join(tmp, f"{tag}.psl")
            subprocess.run([sys.executable, "/root/reference/emtrey.py", "-i", sam, "-o", psl, "-t", "2", "-b", "37"]
                           + mflag, check=True, env=env, cwd=tmp, stdout=subprocess.DEVNULL)
            out[tag + "_psl"] = _digest(psl)
            for primary in (True, False):
                clean = os.path.join(tmp, f"{tag}.clean{int(primary)}.psl")
                S.clean_psl(psl, clean, primary)
                out[f"{tag}_clean_primary{int(primary)}"] = _digest(clean)
    dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "sam_vectors.json")
    json.dump(out, open(dst, "w"), indent=0)
    print("wrote", dst, {k: v["lines"] for k, v in out.items() if isinstance(v, dict)})


if __name__ == "__main__":
    main()
