#!/usr/bin/env python3
"""Module P throughput (SAM -> PSL -> clean PSL -> sorted + locus split), native vs the reference.

usage: python tools/bench_p.py [n_reads] [threads] [--ref] [--gpu]
Input: tests/golden/make_sam_vectors.make_input with n_reads reads (~1.3 records each).  With --ref
(this container only; /root/reference does not exist on the GPU box) the reference's
`python3 emtrey.py -m -t T` + clean_psl + `sort` + get_chromosomes run on the same file under a stand-in
mappy, timed the same way.  Prints one JSON line."""
import contextlib
import importlib.util
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    n_reads = int(args[0]) if args else 100000
    threads = int(args[1]) if len(args) > 1 else 8
    spec = importlib.util.spec_from_file_location("msam", os.path.join(ROOT, "tests", "golden", "make_sam_vectors.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    from mandalorion_amd import psl

    out = {"n_reads": n_reads, "threads": threads}
    with tempfile.TemporaryDirectory(dir="/tmp") as tmp:
        sam = os.path.join(tmp, "in.sam")
        t = time.perf_counter()
        out["records"] = m.make_input(sam, n_reads=n_reads)
        out["gen_s"] = round(time.perf_counter() - t, 2)
        out["sam_mb"] = round(os.path.getsize(sam) / 1e6, 1)
        if "--gpu" in sys.argv:
            # the GPU conversion (sam_kernel.hip) beside the host threads' one: same bytes, both timed
            psl.sam_to_psl(sam, os.path.join(tmp, "g.psl"), mando=True, device=0)  # warm (context, code)
            tg = time.perf_counter()
            psl.sam_to_psl(sam, os.path.join(tmp, "g.psl"), mando=True, device=0)
            out["sam_to_psl_gpu_s"] = round(time.perf_counter() - tg, 3)
        t0 = time.perf_counter()
        psl.sam_to_psl(sam, os.path.join(tmp, "a.psl"), mando=True, threads=threads, device=None)
        t1 = time.perf_counter()
        if "--gpu" in sys.argv:
            out["gpu_equals_host"] = open(os.path.join(tmp, "g.psl"), "rb").read() == open(os.path.join(tmp, "a.psl"), "rb").read()
        psl.clean_psl(os.path.join(tmp, "a.psl"), os.path.join(tmp, "a.clean.psl"), True)
        t2 = time.perf_counter()
        psl.split_loci(os.path.join(tmp, "a.clean.psl"), os.path.join(tmp, "ss"), True, os.path.join(tmp, "a.sorted.psl"),
                       device=None)
        t3 = time.perf_counter()
        if "--gpu" in sys.argv:
            tg = time.perf_counter()
            psl.split_loci(os.path.join(tmp, "a.clean.psl"), os.path.join(tmp, "ssg"), True,
                           os.path.join(tmp, "g.sorted.psl"), device=0)
            out["sort_split_gpu_s"] = round(time.perf_counter() - tg, 3)
            out["split_gpu_equals_host"] = (open(os.path.join(tmp, "g.sorted.psl"), "rb").read() ==
                                            open(os.path.join(tmp, "a.sorted.psl"), "rb").read() and
                                            sorted(os.listdir(os.path.join(tmp, "ssg"))) ==
                                            sorted(os.listdir(os.path.join(tmp, "ss"))))
        out["native_s"] = {"sam_to_psl": round(t1 - t0, 3), "clean": round(t2 - t1, 3), "sort_split": round(t3 - t2, 3)}
        out["native_records_per_s"] = round(out["records"] / (t3 - t0))
        if "--ref" in sys.argv:
            stub = os.path.join(tmp, "stub", "mappy")
            os.makedirs(stub)
            open(os.path.join(stub, "__init__.py"), "w").write(m.STUB)
            env = dict(os.environ, PYTHONPATH=os.path.join(tmp, "stub"), LC_ALL="C")
            sys.path.insert(0, os.path.join(tmp, "stub"))
            sys.path.insert(0, "/root/reference/utils")
            import SpliceDefineConsensus as S

            t0 = time.perf_counter()
            subprocess.run([sys.executable, "/root/reference/emtrey.py", "-i", sam, "-o", os.path.join(tmp, "r.psl"),
                            "-m", "-t", str(threads)], check=True, env=env, cwd=tmp, stdout=subprocess.DEVNULL)
            t1 = time.perf_counter()
            S.clean_psl(os.path.join(tmp, "r.psl"), os.path.join(tmp, "r.clean.psl"), True)
            t2 = time.perf_counter()
            with open(os.path.join(tmp, "r.sorted.psl"), "w") as fh:
                subprocess.run(["sort", "-T", tmp, "-k", "14,14", "-k", "16,17n", os.path.join(tmp, "r.clean.psl")],
                               stdout=fh, check=True, env=env)
            os.makedirs(os.path.join(tmp, "rss"))
            with open(os.devnull, "w") as dn, contextlib.redirect_stdout(dn):
                S.get_chromosomes(os.path.join(tmp, "r.sorted.psl"), os.path.join(tmp, "rss"), [])
            t3 = time.perf_counter()
            out["reference_s"] = {"emtrey": round(t1 - t0, 3), "clean": round(t2 - t1, 3), "sort_split": round(t3 - t2, 3)}
            out["reference_records_per_s"] = round(out["records"] / (t3 - t0))
            same = open(os.path.join(tmp, "r.clean.psl"), "rb").read() == open(os.path.join(tmp, "a.clean.psl"), "rb").read()
            out["identical_clean_psl"] = same
    print(json.dumps(out))


if __name__ == "__main__":
    main()
