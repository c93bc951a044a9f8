"""Dev helper: whole D module on one of the bench's workloads with the stage timeline (cluster chunks on
the host worker thread vs orientation / POA chunks on the GPU).  CHUNKS=<n> fixes the chunk count.
usage: python tools/e2e_timeline.py [workload=config3] [loci]"""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench
from mandalorion_amd import define
wl = sys.argv[1] if len(sys.argv) > 1 else "config3"
n = int(sys.argv[2]) if len(sys.argv) > 2 else bench.WORKLOADS[wl]["loci"]
d = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"mando_bench_{wl}_{n}")
os.makedirs(d, exist_ok=True)
t = time.time(); bench.gen_data(d, bench.WORKLOADS[wl], n, 16); print(f"data {time.time()-t:.1f}s", flush=True)
for nc in [int(x) for x in os.environ.get("CHUNKS", "0").split(",")]:
    define.define_isoforms(d, threads=16, n_chunks=nc)
    st = define.define_isoforms(d, threads=16, n_chunks=nc)
    print(f"== chunks {st['chunks']}: total {st['t_total']:.3f}")
    for k, v in st.items():
        if not isinstance(v, list): print("  ", k, v)
    for x in st["poa_launches"]: print("   poa launch", {k: round(v, 3) if isinstance(v, float) else v for k, v in x.items()})
    for name, a, b in sorted(st["timeline"], key=lambda x: x[1]): print(f"  {name:8s} {a:7.3f} -> {b:7.3f} ({b-a:.3f})")
