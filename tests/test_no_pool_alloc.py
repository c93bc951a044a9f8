"""Guard: no product source allocates from HIP's stream-ordered pool.  On MI355X / ROCm 7.2 a recycled pool
buffer refilled by a completed host-to-device copy still shows a kernel its old bytes
(tools/stale_probe.hip; profiles/r03b_stale_probe.txt), so libmando keeps hipMalloc'd buffers instead."""
import os
import re

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mandalorion_amd", "csrc")


def test_no_stream_ordered_pool_in_product_sources():
    pat = re.compile(r"\bhip(MallocAsync|FreeAsync|MallocFromPoolAsync|MemPoolCreate)\b")
    hits = []
    for f in sorted(os.listdir(CSRC)):
        if f.endswith((".hip", ".cpp", ".h")):
            for n, line in enumerate(open(os.path.join(CSRC, f)), 1):
                code = line.split("//")[0]
                if pat.search(code):
                    hits.append(f"{f}:{n}")
    assert not hits, hits
