"""mando_poa_segments_begin / mando_poa_end (two POA batches in flight on one context, the D driver's
chunk pipeline) against the CPU restatement (oracle/poa_ref.c via oracle.poa): the consensi of every
batch must equal the oracle's whatever order the batches are ended in, a third batch in flight is
refused, and a ticket is ended once."""
from __future__ import annotations

import ctypes

import numpy as np
import pytest

from mandalorion_amd import _lib, poa, synth


class _DevText:
    """The reads' text in a hipMalloc'd device buffer (what mando_cluster_device_text hands the driver)."""

    def __init__(self, data: bytes):
        self.hip = ctypes.CDLL("libamdhip64.so")
        self.p = ctypes.c_void_p()
        assert self.hip.hipMalloc(ctypes.byref(self.p), ctypes.c_size_t(max(len(data), 1))) == 0
        buf = np.frombuffer(data, dtype=np.uint8)
        assert self.hip.hipMemcpy(self.p, ctypes.c_void_p(buf.ctypes.data), ctypes.c_size_t(len(data)), 1) == 0
        self.n = len(data)

    def close(self):
        self.hip.hipFree(self.p)


def _batch(groups, base, rcs):
    """(off, len, rc, grp_off) of groups whose reads sit back to back from `base` in the device text;
    reads with rc set are stored reverse-complemented there (the gather undoes it)."""
    off, ln, rc, grp = [], [], [], [0]
    pos = base
    text = []
    for gi, g in enumerate(groups):
        for ri, s in enumerate(g):
            flip = rcs[(gi + ri) % len(rcs)]
            text.append(synth.revcomp(s) if flip else s)
            off.append(pos)
            ln.append(len(s))
            rc.append(1 if flip else 0)
            pos += len(s)
        grp.append(len(off))
    return ("".join(text).encode(), np.asarray(off, np.int64), np.asarray(ln, np.int32), np.asarray(rc, np.int8),
            np.asarray(grp, np.int64))


@pytest.mark.gpu
def test_two_batches_in_flight_equal_oracle_any_end_order():
    from oracle import poa as opoa

    sets = [synth.read_groups(n, (300, 1500), (3, 14), seed=s)[1] for n, s in ((40, 71), (25, 72), (9, 73))]
    texts, metas, pos = [], [], 0
    for k, groups in enumerate(sets):
        t, off, ln, rc, grp = _batch(groups, pos, (0, 1, 0) if k != 1 else (1,))
        texts.append(t)
        metas.append((off, ln, rc, grp))
        pos += len(t)
    dev = _DevText(b"".join(texts))
    try:
        want = [opoa.consensus_batch(g) for g in sets]
        b0 = poa.poa_segments_begin(dev.p.value, dev.n, *metas[0], slot=7, info={})
        b1 = poa.poa_segments_begin(dev.p.value, dev.n, *metas[1], slot=7, info={})
        with pytest.raises(_lib.MandoError, match="in flight"):
            poa.poa_segments_begin(dev.p.value, dev.n, *metas[2], slot=7)
        outs = {1: b1.end(), 0: b0.end()}  # the later batch first
        with pytest.raises(RuntimeError):
            b0.end()
        b2 = poa.poa_segments_begin(dev.p.value, dev.n, *metas[2], slot=7)
        outs[2] = b2.end()
        for k in range(3):
            cons, cons_off = outs[k]
            raw = cons.tobytes()
            got = [raw[cons_off[i]:cons_off[i + 1]].decode() for i in range(len(sets[k]))]
            assert got == want[k], f"batch {k}"
        assert b0.info["kernel_ms"] > 0 and b0.info["kernel_end_ms"] >= b0.info["kernel_start_ms"]
        # the synchronous entry point on the same context still works between batches
        cons, cons_off = poa.poa_consensus_segments(dev.p.value, dev.n, *metas[0], slot=7)
        raw = cons.tobytes()
        assert [raw[cons_off[i]:cons_off[i + 1]].decode() for i in range(len(sets[0]))] == want[0]
    finally:
        dev.close()


@pytest.mark.gpu
def test_poa_end_rejects_stale_ticket():
    ctx = _lib.context(0, 7)
    cons = np.zeros(16, np.uint8)
    off = np.zeros(2, np.int64)
    rc = ctx.lib.mando_poa_end(ctx.handle, 12345, _lib.ptr(cons), 16, _lib.ptr(off), None, None)
    assert rc == -1
