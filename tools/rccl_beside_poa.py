"""Dev tool: the multi-rank reassembly's RCCL exchange issued while a POA grid holds the GPU.

In an N-rank run each rank places its reads2isoforms.txt blocks (define._place_r2i: mando_alltoallv_bytes,
ncclSend / ncclRecv in one group, staged through device buffers) on its writer thread while its POA launch
runs.  The rehearsal's stand-in communicator cannot show what that costs, because RCCL's kernels need CUs
that the POA grid holds.  On one GPU: a one-rank RCCL communicator (sends to itself: the same staging
copies and one RCCL copy kernel), `mib` MiB exchanged (config 4 at N = 8: ~31 MB of reads2isoforms per rank),
timed alone and while a config-4-shaped POA launch runs; the POA launch is timed with and without the
exchange beside it.  Prints one JSON line.

usage: python tools/rccl_beside_poa.py [mib=32] [groups=20000]
"""
import json
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from mandalorion_amd import _lib, poa, synth  # noqa: E402
from mandalorion_amd.comm import Comm  # noqa: E402


def main():
    mib = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    ng = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
    cctx = _lib.context(0, slot=2)
    comm = Comm(1, 0, device_ctx=cctx)
    if comm.backend != "rccl":
        raise SystemExit(f"backend {comm.backend}")
    blob = np.random.default_rng(1).integers(0, 255, size=mib << 20, dtype=np.uint8)

    def exchange():
        t = time.perf_counter()
        out = comm.alltoallv([blob])
        dt = time.perf_counter() - t
        assert out[0].size == blob.size and np.array_equal(out[0][:4096], blob[:4096])
        return dt

    alone = [exchange() for _ in range(4)][1:]
    s, so, go = synth.fast_groups(ng, (2000, 3600), (25, 25), seed=1)
    pctx = _lib.context(0, 0)

    def run_poa(res):
        t = time.perf_counter()
        poa.poa_consensus_packed(s, so, go, device=0, slot=0)
        res["wall"] = time.perf_counter() - t
        res["kernel_ms"] = pctx.last_kernel_ms()

    base = {}
    run_poa(base)  # warm (workspace allocation)
    base = {}
    run_poa(base)
    beside, runs = [], []
    for k in range(3):
        res = {}
        th = threading.Thread(target=run_poa, args=(res,))
        th.start()
        time.sleep(0.1 + 0.1 * k)  # the grid is running and holds every CU's wave slots
        beside.append(exchange())
        th.join()
        runs.append(res)
    out = {"mib": mib, "poa_groups": ng, "exchange_alone_s": [round(x, 4) for x in alone],
           "exchange_beside_poa_s": [round(x, 4) for x in beside],
           "poa_alone_kernel_ms": round(base["kernel_ms"], 1),
           "poa_with_exchange_kernel_ms": [round(r["kernel_ms"], 1) for r in runs]}
    print(json.dumps(out), flush=True)
    comm.close()


if __name__ == "__main__":
    main()
