#!/usr/bin/env python3
"""Generates tests/golden/cluster_vectors.json from the REFERENCE clustering (run here only).

What it pins (SURVEY.md §8c "Clustering half ... importable here"):
  * per locus, the splice-site peaks `find_peaks` / `make_genome_bins` accept (toWrite rows),
  * per isoform, the ordered read names (`IsoDict`, SpliceDefineConsensus.py:797-868) and the ordered
    abPOA input (`determine_consensus` subsample, :876-926) plus whether `-S` was passed,
  * the exact bytes of Isoform_Consensi.fasta and reads2isoforms.txt written by the unmodified
    defineIsoforms.py (sha256 + the reads2isoforms lines), with a capture-only `abpoa` stand-in that
    returns the first input sequence as the "consensus".
How: the synthetic loci of mandalorion_amd.simdata.fixture_specs() are written to a temp dir; the
reference defineIsoforms.py runs unmodified under a parent that seeds numpy's global RNG (the fork
start method then gives every locus worker the same RNG state, which is what the build replays); mappy
is absent from the image, so a stub module stands in (every read maps once, forward, primary).  The
peaks are taken by calling the reference functions in-process under the same seed.
Nothing from the reference is copied into the repository: only inputs (regenerated from a seed and
checked by hash) and outputs land in the JSON.  The reference does not exist on the GPU box; the tests
only read the JSON.
"""
from __future__ import annotations

import glob
import hashlib
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
REF = "/root/reference"
SEEDS = (0, 7)
PARAMS = dict(cutoff=0.1, splice_site_width=1, minimum_read_count=2, junctions="gtag,gcag,atac,ctac,ctgc,gtat",
              upstream_buffer=10, downstream_buffer=50, white_list_polyA="0")

STUB_MAPPY = '''
class _Hit:
    is_primary = True
    strand = 1
class Aligner:
    def __init__(self, seq=None, preset=None):
        self.seq = seq
    def map(self, seq):
        yield _Hit()
_C = str.maketrans("ACGTNacgtn", "TGCANtgcan")
def revcomp(s):
    return s.translate(_C)[::-1]
def fastx_read(path):
    name, seq = None, []
    for line in open(path):
        line = line.rstrip("\\n")
        if line.startswith(">"):
            if name is not None:
                yield name, "".join(seq), None
            name, seq = line[1:].split()[0], []
        else:
            seq.append(line)
    if name is not None:
        yield name, "".join(seq), None
'''

FAKE_ABPOA = '''#!/bin/bash
# capture-only abpoa: log argv + input names, print the first input record as the consensus
in="${@: -1}"
{ echo "CALL $in"; echo "ARGS $*"; grep '^>' "$in"; echo END; } >> "$ABPOA_LOG"
echo ">Consensus_sequence"
awk 'NR==2{print; exit}' "$in"
'''

RUNNER = '''
import sys, runpy
import numpy as np
seed = int(sys.argv[1])
np.random.seed(seed)
sys.argv = [sys.argv[2]] + sys.argv[3:]
runpy.run_path(sys.argv[0], run_name="__main__")
'''


def sha(path):
    return hashlib.sha256(open(path, "rb").read()).hexdigest()


def peaks_in_process(tmp, roots, bounds, seed):
    """find_peaks / make_genome_bins output per locus, reference functions called in-process."""
    sys.path.insert(0, os.path.join(tmp, "stub"))
    sys.path.insert(0, os.path.join(REF, "utils"))
    import numpy as np
    import SpliceDefineConsensus as S

    out = {}
    left_bounds, right_bounds = bounds
    for root in roots:
        chrom, start, end = root.split("~")
        start, end = int(start), int(end)
        lb = {"5": [], "3": []}
        rb = {"5": [], "3": []}
        for side in ("5", "3"):
            lb[side] = [p for p in left_bounds.get(chrom, {}).get(side, []) if start < p < end]
            rb[side] = [p for p in right_bounds.get(chrom, {}).get(side, []) if start < p < end]
        np.random.seed(seed)
        infile = os.path.join(tmp, "tmp_SS", root + ".psl")
        hl, hr, hc, cs = S.collect_reads(infile, chrom)
        pa = {chrom: {"l": {}, "r": {}}}
        pa, a_l = S.make_genome_bins(lb, "l", chrom, pa, PARAMS["splice_site_width"])
        pa, a_r = S.make_genome_bins(rb, "r", chrom, pa, PARAMS["splice_site_width"])
        junc = PARAMS["junctions"].split(",")
        pa, n_l = S.find_peaks(hl[chrom], True, PARAMS["cutoff"], hc, "l", pa, chrom, cs, start, end,
                               PARAMS["splice_site_width"], PARAMS["minimum_read_count"], junc)
        pa, n_r = S.find_peaks(hr[chrom], False, PARAMS["cutoff"], hc, "r", pa, chrom, cs, start, end,
                               PARAMS["splice_site_width"], PARAMS["minimum_read_count"], junc)
        rows = []
        for tw in (a_l, a_r, n_l, n_r):
            for c, s, e, t, sd, prop in tw:
                rows.append([int(s), int(e), t, sd, prop])
        out[root] = rows
    return out


def parse_abpoa_log(path):
    calls = []
    cur = None
    if not os.path.exists(path):
        return calls
    for line in open(path):
        line = line.rstrip("\n")
        if line.startswith("CALL "):
            cur = {"file": os.path.basename(line[5:]), "names": []}
        elif line.startswith("ARGS "):
            cur["seeding"] = " -S " in f" {line[5:]} "
        elif line.startswith(">"):
            cur["names"].append(line[1:])
        elif line == "END":
            calls.append(cur)
    return calls


def main():
    from mandalorion_amd import simdata

    out = {"params": PARAMS, "seeds": {}, "inputs": {}}
    with tempfile.TemporaryDirectory(dir="/tmp") as tmp:
        loci = simdata.make_dataset(simdata.fixture_specs())
        info = simdata.write_dataset(loci, tmp)
        os.makedirs(os.path.join(tmp, "stub", "mappy"))
        open(os.path.join(tmp, "stub", "mappy", "__init__.py"), "w").write(STUB_MAPPY)
        fake = os.path.join(tmp, "fake_abpoa.sh")
        open(fake, "w").write(FAKE_ABPOA)
        os.chmod(fake, 0o755)
        runner = os.path.join(tmp, "runner.py")
        open(runner, "w").write(RUNNER)
        roots = sorted([l.root for l in loci], key=lambda x: (x.split("~")[0], int(x.split("~")[1])))
        out["inputs"] = {
            "generator": "mandalorion_amd.simdata.make_dataset(fixture_specs(), seed=20250117)",
            "records": info["records"],
            "psl_sha256": {l.root: hashlib.sha256(("\n".join(l.lines) + "\n").encode()).hexdigest() for l in loci},
            "gtf_sha256": sha(info["gtf"]) if info["gtf"] else None,
        }
        gtf = info["gtf"] or "None"
        bounds = ({}, {})
        if info["gtf"]:
            sys.path.insert(0, os.path.join(tmp, "stub"))
            sys.path.insert(0, os.path.join(REF, "utils"))
            import SpliceDefineConsensus as S
            _, lb, rb, _ = S.parse_genome(info["gtf"], {}, {}, PARAMS["white_list_polyA"].split(","))
            bounds = (lb, rb)
        for seed in SEEDS:
            for f in ("Isoform_Consensi.fasta", "reads2isoforms.txt", "abpoa.log"):
                if os.path.exists(os.path.join(tmp, f)):
                    os.remove(os.path.join(tmp, f))
            env = dict(os.environ, PYTHONPATH=os.path.join(tmp, "stub"), ABPOA_LOG=os.path.join(tmp, "abpoa.log"))
            cmd = [sys.executable, "-B", runner, str(seed), os.path.join(REF, "defineIsoforms.py"),
                   "-i", "x", "-p", tmp, "-c", str(PARAMS["cutoff"]), "-g", gtf, "-w", str(PARAMS["splice_site_width"]),
                   "-m", str(PARAMS["minimum_read_count"]), "-W", PARAMS["white_list_polyA"], "-n", "1",
                   "-j", PARAMS["junctions"], "-u", str(PARAMS["upstream_buffer"]), "-d", str(PARAMS["downstream_buffer"]),
                   "-a", fake]
            subprocess.run(cmd, cwd=tmp, env=env, check=True, stdout=subprocess.DEVNULL)
            fasta = os.path.join(tmp, "Isoform_Consensi.fasta")
            r2i = os.path.join(tmp, "reads2isoforms.txt")
            calls = parse_abpoa_log(os.path.join(tmp, "abpoa.log"))
            peaks = peaks_in_process(tmp, roots, bounds, seed)
            out["seeds"][str(seed)] = {
                "isoform_consensi_sha256": sha(fasta),
                "reads2isoforms_sha256": sha(r2i),
                "reads2isoforms": [l.rstrip("\n") for l in open(r2i)],
                "isoform_headers": [l[1:].rstrip("\n") for l in open(fasta) if l.startswith(">")],
                "abpoa_calls": calls,
                "peaks": peaks,
            }
    dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "cluster_vectors.json")
    json.dump(out, open(dst, "w"), indent=1)
    print("wrote", dst)


if __name__ == "__main__":
    main()
