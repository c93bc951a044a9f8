#!/usr/bin/env python3
"""Generates tests/golden/split_vectors.json: the reference's locus split (run here only).

Input: the lines of mandalorion_amd.simdata loci (seed 20250117, some loci placed to overlap on the
same chromosome so that get_chromosomes merges them), shuffled with numpy default_rng(7) into one
clean PSL.  Reference path: `LC_ALL=C sort -k 14,14 -k 16,17n` (Mando.py:343-349, GNU coreutils sort)
then the reference's get_chromosomes (SpliceDefineConsensus.py:442-495, imported with a stub mappy).
Stored: sha256 of the sorted file and of every locus file by name.  Nothing of the reference is copied.
"""
import hashlib
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def make_input(path):
    import numpy as np
    from mandalorion_amd import simdata

    specs = [simdata.LocusSpec(n_reads=6, exons=(2, 5), exon_len=(80, 200), intron_len=(100, 600)) for _ in range(8)]
    specs += [simdata.LocusSpec(n_reads=3, exons=(1, 1), exon_len=(300, 500)) for _ in range(4)]
    # chr1/chr2: neighbouring loci overlap (negative gap) and merge; chr10/chr9: separate loci
    merged = simdata.make_dataset(specs, seed=20250117, chroms=2, gap=-400)
    separate = simdata.make_dataset(specs, seed=20250118, chroms=2, gap=3000)
    lines = [l for loc in merged for l in loc.lines]
    ren = {"\tchr1\t": "\tchr10\t", "\tchr2\t": "\tchr9\t"}
    for loc in separate:
        for l in loc.lines:
            for a, b in ren.items():
                l = l.replace(a, b)
            lines.append(l)
    rng = np.random.default_rng(7)
    rng.shuffle(lines)
    with open(path, "w") as fh:
        fh.write("\n".join(lines) + "\n")
    return len(lines)


def main():
    stub = "class Aligner:\n    pass\ndef revcomp(s):\n    return s\n"
    with tempfile.TemporaryDirectory(dir="/tmp") as tmp:
        os.makedirs(os.path.join(tmp, "stub", "mappy"))
        open(os.path.join(tmp, "stub", "mappy", "__init__.py"), "w").write(stub)
        src = os.path.join(tmp, "clean.psl")
        n = make_input(src)
        srt = os.path.join(tmp, "clean.sorted.psl")
        with open(srt, "w") as out:
            subprocess.run(["sort", "-k", "14,14", "-k", "16,17n", src], stdout=out, check=True,
                           env=dict(os.environ, LC_ALL="C"))
        sys.path.insert(0, os.path.join(tmp, "stub"))
        sys.path.insert(0, "/root/reference/utils")
        import SpliceDefineConsensus as S

        ss = os.path.join(tmp, "tmp_SS")
        os.makedirs(ss)
        S.get_chromosomes(srt, ss, [])
        files = {f: hashlib.sha256(open(os.path.join(ss, f), "rb").read()).hexdigest() for f in sorted(os.listdir(ss))}
        out = {"input": "tests/golden/make_split_vectors.py make_input()", "records": n,
               "sorted_sha256": hashlib.sha256(open(srt, "rb").read()).hexdigest(), "loci": files}
    dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "split_vectors.json")
    json.dump(out, open(dst, "w"), indent=1)
    print("wrote", dst, len(files), "loci")


if __name__ == "__main__":
    main()
