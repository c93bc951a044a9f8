"""Dev tool: page-cache reads of locus files into pageable vs pinned (hipHostMalloc) host memory, by thread
count (the clustering reads into a pinned buffer).  usage: python tools/read_bw_pinned.py <tmp_SS> [files]"""
import ctypes, os, sys, time, threading
import numpy as np

d = sys.argv[1]
fs = sorted(os.path.join(d, f) for f in os.listdir(d))[:int(sys.argv[2]) if len(sys.argv) > 2 else None]
sizes = [os.path.getsize(f) for f in fs]
off = np.concatenate([[0], np.cumsum(sizes)])
total = int(off[-1])
hip = ctypes.CDLL("libamdhip64.so")
p = ctypes.c_void_p()
assert hip.hipHostMalloc(ctypes.byref(p), ctypes.c_size_t(total), 0) == 0
pinned = np.ctypeslib.as_array((ctypes.c_uint8 * total).from_address(p.value))
pageable = np.empty(total, np.uint8)
pageable[:] = 1
pinned[:] = 1


def run(buf, nth):
    mv = memoryview(buf)
    nxt, lock = [0], threading.Lock()

    def work():
        while True:
            with lock:
                i = nxt[0]
                nxt[0] += 1
            if i >= len(fs):
                return
            fd = os.open(fs[i], os.O_RDONLY)
            os.readv(fd, [mv[off[i]:off[i + 1]]])
            os.close(fd)
    t = time.perf_counter()
    th = [threading.Thread(target=work) for _ in range(nth)]
    [x.start() for x in th]
    [x.join() for x in th]
    return time.perf_counter() - t


for nth in (1, 8, 14):
    for name, buf in (("pageable", pageable), ("pinned", pinned)):
        dt = min(run(buf, nth) for _ in range(2))
        print(f"{name:8s} {nth:2d} threads: {total / 1e9:.2f} GB in {dt:.3f} s = {total / 1e9 / dt:.1f} GB/s", flush=True)
