#!/usr/bin/env python3
"""Pins the clustering half of the D module at bench scale against the UNMODIFIED reference itself.

The reference (`/root/reference/defineIsoforms.py` -> `utils/SpliceDefineConsensus.py`) is run here end
to end on one of bench.py's full-size synthetic workloads (config 3: 20,000 loci x 50 reads; config 4:
200,000 loci, ~10M records), under a seeded parent (np.random.seed(0) before the Pool forks, the same
state `define_isoforms(seed=0)` replays), with
  * a stand-in `mappy` whose Aligner.map yields one primary forward hit per read (mappy is absent), and
  * `abpoa` = /bin/true: it writes no consensus, so the reference falls back to its first oriented read
    (SDC:924-925) -- abPOA is absent and the consensus bytes are not what this pins.
What the run pins: `reads2isoforms.txt` and the `>Isoform{k}_{n}` header list.  Both depend only on the
clustering: the reference writes every isoform's `names` (all its reads, SDC:879-883, independent of the
orientation and of the POA) under the global counter of defineIsoforms.py:155-166.  Their sha256 go into
tests/golden/fullsize_hashes.json as `reference_reads2isoforms_sha256` / `reference_headers_sha256` of the
workload's entry; bench.py and tests/test_define_gpu.py compare the GPU run's files against them.

The data are regenerated from the workload's parameters (libmando_synth is a pure function of them), so
the hashes refer to the same bytes bench.py generates on the GPU box.  Nothing from the reference is
copied into the repository: it is run, and only hashes are kept.

With --prefix-loci N the reference runs on the first N loci of the workload (sorted roots, the
reference's own order, defineIsoforms.py:126) -- config 4's 200,000 loci take ~12 h of the reference's
Python on this container's cores, its first 20,000 about 1 h.  Isoforms are numbered in sorted-root
order from 1, so the reference's files over that prefix are byte prefixes of the full run's files: the
entry's `reference_prefix` holds their sizes and sha256 (reads2isoforms.txt bytes, header list).

Usage: python tests/golden/make_reference_fullsize.py config3 [config4 --prefix-loci 20000] [--procs 8]
       [--data-dir /tmp]
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
REF = "/root/reference"
DST = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fullsize_hashes.json")
SEED = 0

STUB_MAPPY = '''
class _Hit:
    is_primary = True
    strand = 1
class Aligner:
    def __init__(self, seq=None, preset=None):
        pass
    def map(self, seq):
        yield _Hit()
def revcomp(s):
    raise AssertionError("forward-only stand-in: revcomp is never reached")
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

RUNNER = '''
import sys, runpy
import numpy as np
np.random.seed(int(sys.argv[1]))
sys.argv = [sys.argv[2]] + sys.argv[3:]
runpy.run_path(sys.argv[0], run_name="__main__")
'''


def sha_file(path: str) -> str:
    h = hashlib.sha256()
    with open(path, "rb") as fh:
        for blk in iter(lambda: fh.read(1 << 24), b""):
            h.update(blk)
    return h.hexdigest()


def headers_sha(fasta: str) -> tuple[str, int]:
    """sha256 over the FASTA's header lines (each with its newline), in file order."""
    h, n = hashlib.sha256(), 0
    with open(fasta, "rb") as fh:
        for line in fh:
            if line.startswith(b">"):
                h.update(line)
                n += 1
    return h.hexdigest(), n


def run_reference(d: str, tools: str, procs: int) -> float:
    env = dict(os.environ, PYTHONPATH=os.path.join(tools, "stub"))
    cmd = [sys.executable, "-B", os.path.join(tools, "runner.py"), str(SEED), os.path.join(REF, "defineIsoforms.py"),
           "-i", "x", "-p", d, "-c", "0.1", "-g", "None", "-w", "1", "-m", "2", "-W", "0", "-n", str(procs),
           "-j", "gtag,gcag,atac,ctac,ctgc,gtat", "-u", "10", "-d", "50", "-a", "/bin/true"]
    t0 = time.perf_counter()
    subprocess.run(cmd, cwd=d, env=env, check=True, stdout=subprocess.DEVNULL)
    return time.perf_counter() - t0


def main():
    import bench

    ap = argparse.ArgumentParser()
    ap.add_argument("workloads", nargs="+")
    ap.add_argument("--procs", type=int, default=os.cpu_count() or 8)
    ap.add_argument("--data-dir", default="/tmp")
    ap.add_argument("--prefix-loci", type=int, default=0)
    a = ap.parse_args()
    with tempfile.TemporaryDirectory(dir="/tmp") as tools:
        os.makedirs(os.path.join(tools, "stub", "mappy"))
        open(os.path.join(tools, "stub", "mappy", "__init__.py"), "w").write(STUB_MAPPY)
        open(os.path.join(tools, "runner.py"), "w").write(RUNNER)
        for name in a.workloads:
            wl = bench.WORKLOADS[name]
            key = f"{name}:{wl['loci']}"
            d = os.path.join(a.data_dir, f"mando_bench_{name}_{wl['loci']}")
            os.makedirs(d, exist_ok=True)
            records = bench.gen_data(d, wl, wl["loci"], a.procs)
            run_dir = d
            if a.prefix_loci:
                run_dir = os.path.join(a.data_dir, f"mando_refprefix_{name}_{a.prefix_loci}")
                sub_records = bench.sample_dir(d, run_dir, a.prefix_loci)
            wall = run_reference(run_dir, tools, a.procs)
            r2_path = os.path.join(run_dir, "reads2isoforms.txt")
            r2i = sha_file(r2_path)
            hsha, n_iso = headers_sha(os.path.join(run_dir, "Isoform_Consensi.fasta"))
            out = json.load(open(DST))
            ent = out.setdefault(key, {})
            if ent.get("records", records) != records:
                raise SystemExit(f"{key}: {records} records generated, the entry says {ent['records']}")
            how = (f"unmodified /root/reference defineIsoforms.py (seeded parent, forward-only mappy stand-in, "
                   f"abpoa=/bin/true) on {a.procs} processes, {wall:.0f} s; tests/golden/make_reference_fullsize.py")
            if a.prefix_loci:
                ent["reference_prefix"] = {"loci": a.prefix_loci, "records": sub_records, "isoforms": n_iso,
                                           "reads2isoforms_bytes": os.path.getsize(r2_path),
                                           "reads2isoforms_sha256": r2i, "headers_sha256": hsha,
                                           "generated_by": how}
            else:
                ent.update(reference_reads2isoforms_sha256=r2i, reference_headers_sha256=hsha,
                           reference_isoforms=n_iso, reference_generated_by=how)
            json.dump(out, open(DST, "w"), indent=1, sort_keys=True)
            print(name, records, "records;", n_iso, "isoforms; reads2isoforms", r2i,
                  "(oracle:", ent.get("reads2isoforms_sha256"), ")", f"{wall:.0f} s",
                  "prefix" if a.prefix_loci else "", flush=True)


if __name__ == "__main__":
    main()
