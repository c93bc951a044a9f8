"""Dev tool: module F's isoform filters (filterIsoforms.process_chr + write_isoforms) timed on the host path
(mando_filter_isoforms, chromosomes in parallel host threads) and with the containment search on the GPU
(mando_filter_isoforms_device), on tests/modf_synth.py inputs of `loci` loci; checks that both write the
same bytes and prints one JSON line.

usage: python tools/bench_f.py [loci=60000] [threads=16]
"""
import json
import os
import shutil
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from mandalorion_amd import modules  # noqa: E402
from tests import modf_synth  # noqa: E402


def main():
    loci = int(sys.argv[1]) if len(sys.argv) > 1 else 60000
    threads = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    d = tempfile.mkdtemp(prefix="mando_f_", dir=os.environ.get("TMPDIR", "/tmp"))
    try:
        t0 = time.perf_counter()
        n_lines = modf_synth.write_inputs(d, n_loci=loci, seed=11, chroms=8)
        t_gen = time.perf_counter() - t0
        print(f"[bench_f] {n_lines} PSL lines in {t_gen:.1f} s", file=sys.stderr, flush=True)
        p = modules.FilterParams.default()
        p.threads = threads
        p.internal_ratio = 0.3
        res, outs = {}, {}
        for label, dev in (("gpu", 0), ("host", None), ("gpu2", 0), ("host2", None)):
            o = os.path.join(d, "out_" + label)
            t = time.perf_counter()
            n = modules.filter_isoforms(p, os.path.join(d, "Isoform_Consensi.fasta"), os.path.join(d, "genome.fa"),
                                        os.path.join(d, "clean.psl"), os.path.join(d, "polyAWhiteList.bed"),
                                        o + ".fa", o + ".psl", o + ".reasons", device=dev)
            res[label] = round(time.perf_counter() - t, 3)
            print(f"[bench_f] {label} {res[label]} s", file=sys.stderr, flush=True)
            outs[label] = (n, open(o + ".psl", "rb").read(), open(o + ".reasons", "rb").read())
        same = outs["gpu"] == outs["host"] == outs["gpu2"] == outs["host2"]
        print(json.dumps({"loci": loci, "psl_lines": n_lines, "kept": outs["gpu"][0], "gen_s": round(t_gen, 1),
                          "host_threads": threads, "host_s": [res["host"], res["host2"]],
                          "gpu_s": [res["gpu"], res["gpu2"]], "outputs_equal": same}))
    finally:
        shutil.rmtree(d, ignore_errors=True)


if __name__ == "__main__":
    main()
