"""Dev tool: page-cache read bandwidth of locus files (the clustering's host reading), by thread count.
usage: python tools/read_bw.py <tmp_SS dir> <threads> [max files]"""
import os, sys, time, threading, numpy as np
d = sys.argv[1]; nth = int(sys.argv[2])
fs = sorted(os.path.join(d, f) for f in os.listdir(d))[:int(sys.argv[3]) if len(sys.argv) > 3 else None]
sizes = [os.path.getsize(f) for f in fs]
off = np.concatenate([[0], np.cumsum(sizes)])
buf = np.empty(int(off[-1]), np.uint8)
mv = memoryview(buf)
nxt = [0]; lock = threading.Lock()
def work():
    while True:
        with lock:
            i = nxt[0]; nxt[0] += 1
        if i >= len(fs): return
        fd = os.open(fs[i], os.O_RDONLY)
        os.readv(fd, [mv[off[i]:off[i+1]]])
        os.close(fd)
for rep in range(2):
    nxt[0] = 0
    t = time.perf_counter()
    th = [threading.Thread(target=work) for _ in range(nth)]
    [x.start() for x in th]; [x.join() for x in th]
    dt = time.perf_counter() - t
    print(nth, "threads: %.2f GB in %.3f s = %.1f GB/s" % (off[-1] / 1e9, dt, off[-1] / 1e9 / dt), flush=True)
