"""Dev helper: orientation kernel time with a share of reverse-complemented reads (D-module shape)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from mandalorion_amd import synth, _lib, orient
n = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
frac = float(sys.argv[2]) if len(sys.argv) > 2 else 0.3
s, so, go = synth.fast_groups(n, (2700, 3300), (25, 25), seed=3, threads=16)
groups = synth.unpack_groups(s, so, go)
rng = np.random.default_rng(1)
groups = [[synth.revcomp(x) if rng.random() < frac else x for x in g] for g in groups]
orient.orient_batch(groups[:100])
t = time.perf_counter()
res = orient.orient_batch(groups)
wall = time.perf_counter() - t
ctx = _lib.context(0)
print(f"groups {n} rev {frac} reads {len(so)-1} wall {wall:.3f}s kernel {ctx.last_kernel_ms():.1f} ms launches {ctx.lib.mando_last_kernel_launches(ctx.handle)}")
