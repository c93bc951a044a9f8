"""Dev helper: per-phase cycle breakdown of the POA kernel (MANDO_PROF=1) on a config-3-shaped batch."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["MANDO_PROF"] = "1"
from mandalorion_amd import synth, poa
n = int(sys.argv[1]) if len(sys.argv) > 1 else 500
lo, hi, dep = (int(os.environ.get(k, d)) for k, d in (("LEN_LO", 2700), ("LEN_HI", 3300), ("DEPTH", 50)))
s, so, go = synth.fast_groups(n, (lo, hi), (dep, dep), seed=1)
groups = synth.unpack_groups(s, so, go)
t = time.time()
out, cells = poa.poa_consensus_batch(groups, return_cells=True)
dt = time.time() - t
from mandalorion_amd import _lib
print(f"groups {n} wall {dt:.3f}s kernel {_lib.context(0).last_kernel_ms():.1f} ms cells {cells.sum():.3e} gcups {cells.sum()/(_lib.context(0).last_kernel_ms()/1e3)/1e9:.2f}")
