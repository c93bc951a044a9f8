"""The D driver's chunk plan and HBM budget (host logic, no GPU): defineIsoforms.py:130-166's per-locus
Pool becomes a few pipelined chunks; the POA workspace budget of a call is derived from its plan
(mando_ctx_set_poa_budget), never from process-global state."""
from __future__ import annotations

import os

import pytest

from mandalorion_amd import define

GB = 1 << 30


@pytest.fixture(autouse=True)
def _clean_env(monkeypatch):
    for k in ("MANDO_CHUNKS",):
        monkeypatch.delenv(k, raising=False)


def test_small_inputs_run_in_one_chunk():
    assert define._chunk_plan(6 * GB, 20000) == (1, None)      # config 3: 6.2 GB of locus text
    assert define._chunk_plan(100 * GB, 7) == (1, None)        # few large loci (SIRV-like)


def test_byte_capped_chunks():
    n, fr = define._chunk_plan(20 * GB, 60000)
    k = -(-20 * GB // define._CHUNK_BYTES)
    assert n == k + 1 and fr == pytest.approx([(0.4 + i) / k for i in range(k)])
    assert fr[0] * 20 * GB < define._CHUNK_BYTES                # the first chunk is the smallest


def test_two_chunks_take_the_first_chunk_fraction(monkeypatch):
    assert define._chunk_plan(GB, 100, n_chunks=2) == (2, [0.3])
    assert define._chunk_plan(GB, 100, fracs=[0.5]) == (2, [0.5])
    monkeypatch.setenv("MANDO_CHUNKS", "2")
    assert define._chunk_plan(GB, 100) == (2, [0.3])
    assert define._chunk_plan(GB, 100, fracs=[0.2, 0.6]) == (3, [0.2, 0.6])
    assert define._chunk_plan(GB, 100, n_chunks=3) == (3, None)  # forced counts other than 2: equal chunks


def test_chunk_count_never_exceeds_loci():
    assert define._chunk_plan(GB, 2, n_chunks=5) == (2, None)


def test_poa_budget_reserves_the_chunks_in_flight():
    total = 288 * 10**9
    one = define.poa_budget(total, [6 * GB])
    many = define.poa_budget(total, [3 * GB] + [8 * GB] * 7)
    assert 4 * GB <= many < one < define._HBM_USABLE * total
    # four pool buffers of the largest chunk, its clustering scratch and gathered reads, 4 GiB of margin
    big = 8 * GB
    want = int(define._HBM_USABLE * total) - 4 * (big + (256 << 20)) - int(
        (define._CLUSTER_SCRATCH_PER_TEXT + 2 * define._GATHERED_PER_TEXT) * big) - 4 * GB
    assert many == want
    assert define.poa_budget(16 * GB, [8 * GB] * 4) == 4 * GB  # never below the floor


def test_no_process_environment_side_effects():
    before = dict(os.environ)
    define._chunk_plan(80 * GB, 200000)
    define.poa_budget(288 * 10**9, [8 * GB] * 10)
    assert dict(os.environ) == before


def test_metrics_line():
    st = {"loci": 10, "records": 500, "isoforms": 12, "poa_groups": 11, "poa_reads": 400, "t_total": 2.0,
          "t_cluster": 0.5, "chunks": 1,
          "poa_launches": [{"cells": 8 * 10**9, "read_bytes": 10**6, "cons_bytes": 10**4, "kernel_ms": 1000.0,
                            "launches": 2, "reads": 400}]}
    m = define.metrics(st)
    assert m["records_per_s_rank0"] == 250 and m["gcups"] == pytest.approx(8.0)
    assert m["poa_algorithmic_GBps"] == pytest.approx((8 * 10**9 + 10**6 + 10**4) / 1e9)
    assert m["poa_hbm_roofline_frac"] == pytest.approx(m["poa_algorithmic_GBps"] / 8000.0)
    assert define.metrics({"t_total": 1.0, "records": 0})["gcups"] is None


def _py_outputs(order, mem_off, counter0, cons, names):
    """defineIsoforms.py:155-166 written the plain way: one f-string per isoform and per member."""
    comp = bytes.maketrans(b"ACGTNacgtn", b"TGCANtgcan")
    fa, r2 = [], []
    for i, g in enumerate(order):
        lab = f"Isoform{counter0 + 1 + i}_{mem_off[g + 1] - mem_off[g]}".encode()
        srcs, sel, st, ln, rc = cons
        c = bytes(srcs[sel[g]][st[g]:st[g] + ln[g]])
        fa.append(b">" + lab + b"\n" + (c[::-1].translate(comp) if rc[g] else c) + b"\n")
        srcs, sel, st, ln = names
        for j in range(mem_off[g], mem_off[g + 1]):
            r2.append(bytes(srcs[sel[j]][st[j]:st[j] + ln[j]]) + b"\t" + lab + b"\n")
    return b"".join(fa), b"".join(r2)


@pytest.mark.parametrize("n_iso,counter0", [(0, 0), (1, 0), (37, 9), (20000, 99995)])
def test_format_outputs_matches_the_per_isoform_loop(n_iso, counter0):
    import numpy as np

    from mandalorion_amd import _lib

    rng = np.random.default_rng(n_iso)
    text = [rng.choice(np.frombuffer(b"ACGTNacgtn", np.uint8), 5000), rng.choice(np.frombuffer(b"ACGT", np.uint8), 300)]
    m = rng.integers(0, 12, n_iso)
    mem_off = np.zeros(n_iso + 1, np.int64)
    np.cumsum(m, out=mem_off[1:])
    c_sel = rng.integers(0, 2, n_iso).astype(np.int16)
    c_len = rng.integers(0, 200, n_iso)
    c_start = np.array([rng.integers(0, len(text[s]) - ln + 1) for s, ln in zip(c_sel, c_len)], np.int64)
    c_rc = rng.integers(0, 2, n_iso).astype(np.int8)
    nm = int(mem_off[-1])
    n_sel = rng.integers(0, 2, nm).astype(np.int16)
    n_len = rng.integers(1, 40, nm)
    n_start = np.array([rng.integers(0, len(text[s]) - ln + 1) for s, ln in zip(n_sel, n_len)], np.int64)
    order = rng.permutation(n_iso)
    cons = (text, c_sel, c_start, c_len, c_rc)
    names = (text, n_sel, n_start, n_len)
    fa, r2 = _lib.format_outputs(order, mem_off, counter0, cons, names, threads=4)
    want = _py_outputs(order, mem_off, counter0, cons, names)
    assert fa.tobytes() == want[0] and r2.tobytes() == want[1]
    fa2, none = _lib.format_outputs(order, mem_off, counter0, cons, None)
    assert none is None and fa2.tobytes() == want[0]
    none, r22 = _lib.format_outputs(order, mem_off, counter0, None, names, threads=1)
    assert none is None and r22.tobytes() == want[1]


def test_write_big_appends_in_order(tmp_path):
    import numpy as np

    a = (np.arange(5 << 20) % 251).astype(np.uint8)
    p = tmp_path / "out"
    with open(p, "wb") as fh:
        fh.write(b"head")
        define._write_big(fh, a, piece=1 << 20)   # 5 parallel pwrite pieces
        fh.write(b"tail")
    got = p.read_bytes()
    assert got == b"head" + a.tobytes() + b"tail"


def test_shard_plan_balances_and_is_lpt_for_the_heaviest():
    import numpy as np

    rng = np.random.default_rng(3)
    cost = rng.uniform(1, 100, 5000) ** 2
    owner = define._lpt_owner(cost, 8, head=16)
    load = np.bincount(owner, weights=cost, minlength=8)
    assert load.max() / load.mean() < 1.001
    # the heaviest 8 go to 8 different ranks, the 9th to the least-loaded of them
    top = np.argsort(-cost, kind="stable")
    assert sorted(owner[top[:8]]) == list(range(8))
    assert owner[top[8]] == owner[top[7]]
    assert define._lpt_owner(np.array([5.0, 1.0]), 4).tolist() == [0, 1]
    assert define._lpt_owner(np.zeros(0), 3).size == 0


@pytest.mark.parametrize("flags", ["rw", "wo"])
def test_write_blocks_places_every_block(tmp_path, flags):
    """mando_write_blocks: blocks of a buffer land at their file offsets (through a shared mapping when the
    descriptor is read-write, pwrite() otherwise), neighbouring blocks coalesced, empty ones skipped."""
    import numpy as np

    from mandalorion_amd import _lib

    rng = np.random.default_rng(3)
    n = 5000
    ln = rng.integers(0, 3000, n)
    dst = np.zeros(n, np.int64)
    np.cumsum(ln[:-1], out=dst[1:])
    perm = rng.permutation(n)                       # the buffer holds the blocks in another order
    src = np.zeros(n, np.int64)
    np.cumsum(ln[perm][:-1], out=src[1:])
    src_of = np.empty(n, np.int64)
    src_of[perm] = src
    want = rng.integers(0, 256, int(ln.sum()), dtype=np.uint8)
    buf = np.empty_like(want)
    for i in range(n):
        buf[src_of[i]:src_of[i] + ln[i]] = want[dst[i]:dst[i] + ln[i]]
    p = tmp_path / "f"
    with open(p, "wb") as fh:
        fh.write(b"\xee" * (len(want) + 10))          # stale bytes everywhere
    fd = os.open(p, os.O_RDWR if flags == "rw" else os.O_WRONLY)
    try:
        os.ftruncate(fd, len(want))
        _lib.write_blocks(fd, buf, src_of, dst, ln, threads=4)
    finally:
        os.close(fd)
    assert p.read_bytes() == want.tobytes()
