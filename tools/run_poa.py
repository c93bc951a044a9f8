"""Dev helper: one POA batch on a config-3-shaped sample (for rocprofv3 counter passes)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mandalorion_amd import synth, poa, _lib
n = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
s, so, go = synth.fast_groups(n, (2700, 3300), (50, 50), seed=1, threads=16)
groups = synth.unpack_groups(s, so, go)
out, cells = poa.poa_consensus_batch(groups, return_cells=True)
ms = _lib.context(0).last_kernel_ms()
print(f"groups {n} kernel {ms:.1f} ms gcups {cells.sum()/(ms/1e3)/1e9:.2f}")
