"""Repeat check: the SIRV-like loci clustered N times in one process on the GPU; every call must give the
restatement's 67 isoforms with all loci ok (catches stale device buffers between calls).
usage: python tools/cluster_repeat.py <label> <N>"""
import os, sys, json
sys.path.insert(0, os.getcwd())
import numpy as np
from mandalorion_amd import synth, cluster, define
G = json.load(open("tests/golden/define_vectors.json"))
spec = dict(G["datasets"]["sirv_like"]["synth"]); n = spec.pop("n_loci")
d = "/tmp/sirvdbg"
if not os.path.exists(d): synth.write_loci(d + "/tmp_SS", n, threads=8, **spec)
roots = define._roots(d + "/tmp_SS"); paths = [d + "/tmp_SS/" + r + ".psl" for r in roots]; ch = [r.split("~")[0] for r in roots]
bad = 0
for rep in range(int(sys.argv[2])):
    try:
        g = cluster.cluster_loci(paths, ch, threads=8)
        ok = (g.locus_status == 0).all() and g.n_isoforms == 67
        g.close()
    except Exception as e:
        ok = False
    bad += not ok
print(sys.argv[1], "failures", bad, "of", sys.argv[2], flush=True)
