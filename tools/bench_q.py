"""Dev tool: module Q (assignReadsToIsoforms.py) timed on the host path (mando_quantify) and on the GPU
path (mando_quantify_device) on synthetic inputs: `reads` reads of 100 nt in two FASTA files, one
reads2isoforms line per read over `isoforms` isoforms, every isoform in the filtered PSL.  Checks that
both write the same tables and prints one JSON line.

usage: python tools/bench_q.py [reads=4000000] [isoforms=100000]
"""
import json
import os
import shutil
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from mandalorion_amd import modules  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4_000_000
    ni = int(sys.argv[2]) if len(sys.argv) > 2 else 100_000
    d = tempfile.mkdtemp(prefix="mando_q_", dir=os.environ.get("TMPDIR", "/tmp"))
    try:
        rng = np.random.default_rng(7)
        seq = "ACGT" * 25
        t0 = time.perf_counter()
        names = [f"m64011_{i:09d}/ccs" for i in range(n)]
        half = n // 2
        for path, part in (("a.fasta", names[:half]), ("b.fasta", names[half:])):
            with open(os.path.join(d, path), "w") as fh:
                fh.write("".join(f">{nm}\n{seq}\n" for nm in part))
        iso = [f"Isoform{k}_{k % 97 + 1}" for k in range(ni)]
        which = rng.integers(0, ni, size=n)
        with open(os.path.join(d, "reads2isoforms.txt"), "w") as fh:
            fh.write("".join(f"{nm}\t{iso[w]}\n" for nm, w in zip(names, which)))
        used = sorted(set(which.tolist()))
        with open(os.path.join(d, "Isoforms.filtered.clean.psl"), "w") as fh:
            pad = "\t".join(["0"] * 11)
            fh.write("".join(f"0\t0\t0\t0\t0\t0\t0\t0\t+\t{iso[k]}\t{pad}\n" for k in used))
        t_gen = time.perf_counter() - t0
        files = [os.path.join(d, "a.fasta"), os.path.join(d, "b.fasta")]
        out = {}
        for label, dev in (("host", None), ("gpu", 0), ("gpu2", 0), ("host2", None)):
            t = time.perf_counter()
            modules.quantify(d, files, device=dev)
            out[label] = round(time.perf_counter() - t, 3)
            q = open(os.path.join(d, "Isoforms.filtered.clean.quant"), "rb").read()
            tp = open(os.path.join(d, "Isoforms.filtered.clean.tpm"), "rb").read()
            out[label + "_sha"] = (len(q), hash(q), hash(tp))
        same = out["host_sha"] == out["gpu_sha"] == out["gpu2_sha"] == out["host2_sha"]
        print(json.dumps({"reads": n, "isoforms_listed": len(used), "gen_s": round(t_gen, 1),
                          "host_s": [out["host"], out["host2"]], "gpu_s": [out["gpu"], out["gpu2"]],
                          "tables_equal": same}))
    finally:
        shutil.rmtree(d, ignore_errors=True)


if __name__ == "__main__":
    main()
