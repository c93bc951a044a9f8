"""Dev tool: the clustering call alone (no POA beside it) on a bench data set's loci, N at a time, with
MANDO_CL_TIME's split (read + copy, kernels).  usage: python tools/cluster_only.py <data dir> <N> [threads]
[calls]: `calls` consecutive calls over loci [0, N), [N, 2N), ... (default 3 calls over the first N)"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["MANDO_CL_TIME"] = "1"
from mandalorion_amd import cluster, define  # noqa: E402

d, n = sys.argv[1], int(sys.argv[2])
threads = int(sys.argv[3]) if len(sys.argv) > 3 else 14
tmp = os.path.join(d, "tmp_SS")
calls = int(sys.argv[4]) if len(sys.argv) > 4 else 0
roots = define._roots(tmp)
for rep in range(calls or 3):
    sel = roots[rep * n:(rep + 1) * n] if calls else roots[:n]
    paths = [os.path.join(tmp, r + ".psl") for r in sel]
    chroms = [r.split("~")[0] for r in sel]
    t = time.perf_counter()
    res = cluster.cluster_loci(paths, chroms, threads=threads)
    print(f"rep {rep}: {len(paths)} loci, {time.perf_counter() - t:.3f} s", file=sys.stderr, flush=True)
    res.close()
