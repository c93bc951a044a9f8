#!/usr/bin/env python3
"""Generates tests/golden/define_vectors.json: the UNMODIFIED reference D module (defineIsoforms.py ->
SpliceDefineConsensus.py) run here end to end with REAL consensi and REAL orientation decisions.

Round 1's cluster_vectors.json pinned the driver's plumbing with a stub consensus (= first read) and a
stub mappy that maps every read forward, so the reference writer never saw a reverse-strand read, the
duplicate-primary rebinding, the `-S` branch or a real consensus.  Here:
  * mappy (absent from the image) is a stand-in whose Aligner(seq=first).map(seq) yields the primary
    hits of oracle/orient_ref.c (our C restatement of minimap2 map-ont: strand per primary hit) —
    reverse-strand reads are flipped by the reference's own code (SDC:902-907, mp.revcomp);
  * `abpoa` (absent) is a stand-in that runs oracle/poa_ref.c (our C restatement of abPOA v1.4.1,
    including the `-S` window partition) on the FASTA the reference writes, honouring its argv;
  * the data are libmando_synth loci with 35 % '-' strand records, plus a few loci of 8-11 kb reads
    whose median length crosses the reference's 8000 nt `-S` threshold (SDC:914-919).
The reference's own writer (defineIsoforms.py:155-168) produces the files; their sha256 (and the
abPOA argv per isoform) land in the JSON.  The GPU driver (mandalorion_amd.define + the HIP kernels)
must reproduce both files byte for byte (tests/test_define_gpu.py); the host driver with the oracle
functions injected must too (tests/test_define_ref.py).  What this pins: clustering, RNG replay,
subsample order, rebinding, revcomp, the <=2 and empty-consensus fallbacks, `-S` selection and the
writer — against the reference's code.  What it cannot pin: mappy and abPOA themselves (absent; parity
of the restatements with them stays unpinned).
Nothing from the reference is copied into the repository; the reference is run, not read into it.
"""
from __future__ import annotations

import hashlib
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
REF = "/root/reference"
DST = os.path.join(os.path.dirname(os.path.abspath(__file__)), "define_vectors.json")
SEED = 0
PARAMS = dict(cutoff=0.1, splice_site_width=1, minimum_read_count=2, junctions="gtag,gcag,atac,ctac,ctgc,gtat",
              upstream_buffer=10, downstream_buffer=50, white_list_polyA="0")
# datasets: (name, synth.write_loci kwargs)
DATASETS = {
    "r2c2_rev": dict(n_loci=48, reads=(6, 40), exons=(4, 10), exon_len=(150, 400), rev_frac=0.35, seed=4242),
    "deep": dict(n_loci=6, reads=(110, 170), exons=(3, 6), exon_len=(120, 300), rev_frac=0.4, seed=99),
    # BASELINE configs[1] shape: SIRV-like, 7 genes x ~10 isoforms, ~50k reads (~7,000 per locus)
    "sirv_like": dict(n_loci=7, reads=(6500, 7500), exons=(10, 14), exon_len=(60, 200), isoforms=(9, 11),
                      rev_frac=0.3, seed=20250117),
    "long_seeded": dict(n_loci=3, reads=(5, 9), exons=(8, 10), exon_len=(950, 1150), rev_frac=0.3, seed=777),
    # BASELINE configs[0]: 100 synthetic loci x 5 reads x ~1 kb (the reference's CPU plumbing case,
    # Mando.py -M D -> defineIsoforms.py with Mando.py:382-399's argv)
    "config1": dict(n_loci=100, reads=(5, 5), exons=(3, 5), exon_len=(200, 300), isoforms=(1, 1), rev_frac=0.3,
                    seed=1001),
}

STUB_MAPPY = '''
import sys
sys.path.insert(0, {root!r})
from oracle import orient as _o
class _Hit:
    is_primary = True
    def __init__(self, s):
        self.strand = s
class Aligner:
    def __init__(self, seq=None, preset=None):
        self.seq = seq
    def map(self, seq):
        for s in _o.orient_batch([[self.seq, seq]], max_hits=8)[0][1]:
            yield _Hit(int(s))
_C = bytes.maketrans(b"ACGTURYKMBVDHSWNacgturykmbvdhswn", b"TGCAAYRMKVBHDSWNtgcaayrmkvbhdswn")
def revcomp(s):
    return s.encode().translate(_C)[::-1].decode()
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

ORACLE_ABPOA = '''#!{py}
import os, sys
sys.path.insert(0, {root!r})
from oracle import poa as _p
argv = sys.argv[1:]
seeding = "-S" in argv
path = argv[-1]
names, seqs, cur = [], [], None
for line in open(path):
    line = line.rstrip("\\n")
    if line.startswith(">"):
        names.append(line[1:]); seqs.append("")
    else:
        seqs[-1] += line
with open(os.environ["ABPOA_LOG"], "a") as fh:
    fh.write("CALL %s %d %s\\n" % (os.path.basename(path), int(seeding), " ".join(names)))
if seqs:
    print(">Consensus_sequence")
    print(_p.consensus_batch([seqs], seeding=[seeding])[0])
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


def write_dataset(d: str, kw: dict) -> dict:
    from mandalorion_amd import synth

    kw = dict(kw)
    n = kw.pop("n_loci")
    recs = synth.write_loci(os.path.join(d, "tmp_SS"), n, threads=4, **kw)
    files = sorted(os.listdir(os.path.join(d, "tmp_SS")))
    return {"records": recs,
            "psl_sha256": {f: sha(os.path.join(d, "tmp_SS", f)) for f in files}}


def run_reference(d: str, tools: str) -> dict:
    for f in ("Isoform_Consensi.fasta", "reads2isoforms.txt", "abpoa.log"):
        if os.path.exists(os.path.join(d, f)):
            os.remove(os.path.join(d, f))
    env = dict(os.environ, PYTHONPATH=os.path.join(tools, "stub"), ABPOA_LOG=os.path.join(d, "abpoa.log"))
    cmd = [sys.executable, "-B", os.path.join(tools, "runner.py"), str(SEED), os.path.join(REF, "defineIsoforms.py"),
           "-i", "x", "-p", d, "-c", str(PARAMS["cutoff"]), "-g", "None", "-w", str(PARAMS["splice_site_width"]),
           "-m", str(PARAMS["minimum_read_count"]), "-W", PARAMS["white_list_polyA"], "-n", "8",
           "-j", PARAMS["junctions"], "-u", str(PARAMS["upstream_buffer"]), "-d", str(PARAMS["downstream_buffer"]),
           "-a", os.path.join(tools, "abpoa")]
    subprocess.run(cmd, cwd=d, env=env, check=True, stdout=subprocess.DEVNULL)
    fasta, r2i = os.path.join(d, "Isoform_Consensi.fasta"), os.path.join(d, "reads2isoforms.txt")
    calls = []
    for line in open(os.path.join(d, "abpoa.log")):
        _, f, s, *names = line.split()
        calls.append({"n_reads": len(names), "seeding": s == "1"})
    # flipped reads seen by the reference writer: a read whose name appears in an abpoa call with its
    # sequence reverse-complemented is not recorded here; the count of '-' records is in the inputs
    return {"isoform_consensi_sha256": sha(fasta), "reads2isoforms_sha256": sha(r2i),
            "isoform_headers": [l[1:].rstrip("\n") for l in open(fasta) if l.startswith(">")],
            "n_abpoa_calls": len(calls), "n_seeded_calls": sum(c["seeding"] for c in calls),
            "fasta_bytes": os.path.getsize(fasta)}


def main():
    out = {"params": PARAMS, "seed": SEED, "datasets": {}}
    with tempfile.TemporaryDirectory(dir="/tmp") as tmp:
        tools = os.path.join(tmp, "tools")
        os.makedirs(os.path.join(tools, "stub", "mappy"))
        open(os.path.join(tools, "stub", "mappy", "__init__.py"), "w").write(STUB_MAPPY.format(root=ROOT))
        ab = os.path.join(tools, "abpoa")
        open(ab, "w").write(ORACLE_ABPOA.format(py=sys.executable, root=ROOT))
        os.chmod(ab, 0o755)
        open(os.path.join(tools, "runner.py"), "w").write(RUNNER)
        only = sys.argv[1:] or list(DATASETS)
        if os.path.exists(DST):  # keep datasets not regenerated in this run
            out["datasets"] = {k: v for k, v in json.load(open(DST))["datasets"].items() if k not in only}
        for name, kw in DATASETS.items():
            if name not in only:
                continue
            d = os.path.join(tmp, name)
            os.makedirs(d)
            inputs = write_dataset(d, kw)
            res = run_reference(d, tools)
            out["datasets"][name] = {"synth": kw, "inputs": inputs, "reference": res}
            print(name, inputs["records"], "records;", res["n_abpoa_calls"], "abpoa calls,",
                  res["n_seeded_calls"], "with -S")
    out["datasets"] = {k: out["datasets"][k] for k in DATASETS if k in out["datasets"]}
    json.dump(out, open(DST, "w"), indent=1)
    print("wrote", DST)


if __name__ == "__main__":
    main()
