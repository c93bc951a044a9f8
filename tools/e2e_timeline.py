"""Dev helper: whole D module on N synthetic config-3 loci with the stage timeline (cluster chunks on
the host worker thread vs orientation+POA chunks on the GPU)."""
import os, sys, shutil, tempfile, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mandalorion_amd import define, synth
n = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
d = tempfile.mkdtemp(prefix="mando_tl_", dir=os.environ.get("TMPDIR", "/tmp"))
try:
    t = time.time(); synth.write_loci(os.path.join(d, "tmp_SS"), n, threads=16); print(f"write {time.time()-t:.1f}s")
    nc = int(os.environ.get("CHUNKS", "0"))
    define.define_isoforms(d, threads=16, n_chunks=nc)
    st = define.define_isoforms(d, threads=16, n_chunks=nc)
    for k, v in st.items():
        if k != "timeline": print(k, v)
    for name, a, b in sorted(st["timeline"], key=lambda x: x[1]): print(f"  {name:8s} {a:7.3f} -> {b:7.3f} ({b-a:.3f})")
finally:
    shutil.rmtree(d, ignore_errors=True)
