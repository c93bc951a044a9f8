# Dev tool: 8 processes place ~1 GB of blocks into one file through mando_write_blocks at once, with the
# roots interleaved (the snake plan), in contiguous ranges, or dealt in blocks of B roots.
import os, sys, time, numpy as np, multiprocessing as mp
sys.path.insert(0, "/root/repo")
from mandalorion_amd import _lib
N, NB = 8, 200000
rng = np.random.default_rng(1)
sizes = rng.integers(2000, 8000, NB).astype(np.int64)   # ~1 GB of FASTA blocks
off = np.concatenate([[0], np.cumsum(sizes)])
total = int(off[-1])
def run(rank, mode, path, q, barrier):
    if mode == "scatter":
        idx = np.arange(rank, NB, N)            # interleaved roots (LPT-like)
    elif mode.startswith("blk"):
        B = int(mode[3:]); b = np.arange(NB) // B
        idx = np.nonzero(b % N == rank)[0]
    else:
        idx = np.arange(rank * NB // N, (rank + 1) * NB // N)   # contiguous range
    ln = sizes[idx]; src = np.concatenate([[0], np.cumsum(ln)[:-1]])
    buf = np.full(int(ln.sum()), 65 + rank, np.uint8)
    fd = os.open(path, os.O_RDWR)
    barrier.wait()
    t = time.perf_counter()
    _lib.write_blocks(fd, buf, src, off[idx], ln, threads=2)
    q.put(time.perf_counter() - t)
    os.close(fd)
for mode in ("scatter", "contig", "blk256", "blk1024", "blk64", "contig", "blk256"):
    path = "/tmp/place_test.bin"
    fd = os.open(path, os.O_RDWR | os.O_CREAT | os.O_TRUNC, 0o644); os.ftruncate(fd, total); os.close(fd)
    q = mp.Queue(); b = mp.Barrier(N)
    ps = [mp.Process(target=run, args=(r, mode, path, q, b)) for r in range(N)]
    [p.start() for p in ps]; [p.join() for p in ps]
    ts = [q.get() for _ in range(N)]
    print(mode, "max %.3f s" % max(ts), "GB %.2f" % (total / 1e9))
    os.unlink(path)
