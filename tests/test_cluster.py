"""Clustering + D-driver parity against the reference's own outputs (tests/golden/cluster_vectors.json).

The fixtures were produced by the unmodified reference defineIsoforms.py (seeded parent, stub mappy,
capture-only abpoa that answers with the first input sequence) on the synthetic loci of
mandalorion_amd.simdata.fixture_specs(); see tests/golden/make_cluster_vectors.py.  Here the same loci
are regenerated (hash-checked), clustered, and run through the D driver with the same two stand-ins
injected (every read one forward primary hit; consensus = first input sequence), so the written files
must be byte-identical to the reference's.
CPU: the clustering restatement (oracle/cluster_ref.cpp) against the fixtures — this pins the oracle.
GPU: the HIP clustering kernels (libmando mando_cluster_loci) against the same fixtures.
"""
from __future__ import annotations

import hashlib
import json
import os
import socket

import pytest

import numpy as np

from mandalorion_amd import _lib, cluster, define, gtf, simdata
from oracle import cluster as ocl

# (clustering function, pytest marks): the oracle on CPU, the HIP kernels on the GPU
CLUSTERERS = [pytest.param("oracle", id="oracle"), pytest.param("gpu", id="gpu", marks=pytest.mark.gpu)]


def _cl(kind):
    return ocl.cluster_loci if kind == "oracle" else cluster.cluster_loci

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "cluster_vectors.json")))
P = GOLD["params"]


@pytest.fixture(scope="module")
def dataset(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("dmod"))
    loci = simdata.make_dataset(simdata.fixture_specs())
    info = simdata.write_dataset(loci, d)
    for l in loci:
        h = hashlib.sha256(("\n".join(l.lines) + "\n").encode()).hexdigest()
        assert GOLD["inputs"]["psl_sha256"][l.root] == h, "synthetic generator drifted from the fixture"
    roots = sorted([l.root for l in loci], key=lambda x: (x.split("~")[0], int(x.split("~")[1])))
    return d, roots, info


def _stub_orient(seqs, seq_off, grp_off):
    """mappy stand-in of the fixture run: every read one forward primary hit."""
    n = len(seq_off) - 1
    return np.ones((n, 1), dtype=np.int8), np.ones(n, dtype=np.int32)


def _first_of_groups(seqs, seq_off, grp_off):
    """abpoa stand-in of the fixture run: the group's first input sequence."""
    first = grp_off[:-1]
    return _lib.pack_segments([seqs], seq_off[first], seq_off[first + 1] - seq_off[first])


def _stub_consensus(seqs, seq_off, grp_off, seeding):
    _stub_consensus.calls = [(int(grp_off[i + 1] - grp_off[i]), bool(seeding[i])) for i in range(len(grp_off) - 1)]
    return _first_of_groups(seqs, seq_off, grp_off)


def _ann(info, roots):
    _, lb, rb, _ = gtf.parse_genome(info["gtf"], P["white_list_polyA"].split(","))
    return [gtf.locus_bounds(lb, rb, r.split("~")[0], int(r.split("~")[1]), int(r.split("~")[2])) for r in roots]


@pytest.mark.parametrize("kind", CLUSTERERS)
@pytest.mark.parametrize("seed", [0, 7])
def test_peaks_and_isoforms_match_reference(dataset, seed, kind):
    d, roots, info = dataset
    exp = GOLD["seeds"][str(seed)]
    res = _cl(kind)([os.path.join(d, "tmp_SS", r + ".psl") for r in roots], [r.split("~")[0] for r in roots],
                               ann=_ann(info, roots), seed=seed, threads=4)
    assert (res.locus_status == 0).all()
    for li, r in enumerate(roots):
        got = [[p.start, p.end, p.type, p.side, p.prop_str] for p in res.peaks(li)]
        assert got == exp["peaks"][r], r
    lines, calls, k = [], [], 0
    for i in range(res.n_isoforms):
        k += 1
        mem = res.members(i)
        nm = f"Isoform{k}_{len(mem)}"
        lines += [f"{res.name(m)}\t{nm}" for m in mem]
        sub = res.subsample(i)
        if len(sub) > 2:
            calls.append([res.name(m) for m in sub])
    assert lines == exp["reads2isoforms"]
    assert calls == [c["names"] for c in exp["abpoa_calls"]]


@pytest.mark.parametrize("kind", CLUSTERERS)
@pytest.mark.parametrize("seed,chunks", [(0, 1), (7, 1), (0, 3)])
def test_define_driver_files_byte_identical(dataset, seed, chunks, kind, tmp_path):
    d, roots, info = dataset
    exp = GOLD["seeds"][str(seed)]
    stats = define.define_isoforms(d, cutoff=P["cutoff"], genome_file=info["gtf"], splice_site_width=P["splice_site_width"],
                                   minimum_read_count=P["minimum_read_count"], white_list_polyA=P["white_list_polyA"].split(","),
                                   threads=2, junctions=P["junctions"], upstream_buffer=P["upstream_buffer"],
                                   downstream_buffer=P["downstream_buffer"], seed=seed, orient_fn=_stub_orient,
                                   consensus_fn=_stub_consensus, n_chunks=chunks,
                                   cluster_fn=ocl.cluster_loci if kind == "oracle" else None)
    assert stats["chunks"] == chunks
    sha = lambda f: hashlib.sha256(open(os.path.join(d, f), "rb").read()).hexdigest()
    assert sha("Isoform_Consensi.fasta") == exp["isoform_consensi_sha256"]
    assert sha("reads2isoforms.txt") == exp["reads2isoforms_sha256"]
    assert stats["poa_groups"] == len(exp["abpoa_calls"])
    if chunks == 1:
        assert [s for _, s in _stub_consensus.calls] == [c["seeding"] for c in exp["abpoa_calls"]]
        assert [n for n, _ in _stub_consensus.calls] == [len(c["names"]) for c in exp["abpoa_calls"]]


def test_rebinding_and_fallbacks(dataset):
    """determine_consensus quirks (SDC:895-926): a read with two primary hits is written twice (the
    second hit's orientation applies to the already re-bound sequence); <=2 oriented reads -> the first;
    zero -> IndexError."""
    d, roots, _ = dataset
    res = ocl.cluster_loci([os.path.join(d, "tmp_SS", roots[0] + ".psl")], [roots[0].split("~")[0]], seed=0)
    sub = res.subsample(0)
    n = len(sub)
    assert n >= 3 and res.n_isoforms >= 1
    nsub = int(res.sub_off[-1])
    s0 = res.seq(int(sub[0]))

    def run(hits_rows):
        hits = np.zeros((nsub, 4), dtype=np.int8)
        nh = np.ones(nsub, dtype=np.int32)
        for r, row in enumerate(hits_rows):
            hits[r, :len(row)] = row
            nh[r] = len(row)
        hits[len(hits_rows):, 0] = 1
        return define.Assembly(res, hits, nh)

    # read 0 maps twice (+, -), the others not at all -> [s0, revcomp(s0)] -> direct consensus = s0
    a = run([[1, -1]] + [[] for _ in sub[1:]])
    assert bool(a.direct[0]) and a.n_emit[0] == 2 and list(a.e_sign[:2]) == [1, -1]
    # read 0 on '-': the first sequence is its reverse complement; everything goes to the POA
    a = run([[-1]] + [[1] for _ in sub[1:]])
    assert not a.direct[0]
    seqs, off, grp = a.poa_input()
    assert bytes(seqs[off[0]:off[1]]).decode() == define.revcomp(s0) and grp[1] == n
    # second hit of a '-' read flips it back (re-binding): [-1, -1] -> revcomp, then forward again
    a = run([[-1, -1]] + [[1] for _ in sub[1:]])
    seqs, off, _ = a.poa_input()
    assert bytes(seqs[off[0]:off[1]]).decode() == define.revcomp(s0)
    assert bytes(seqs[off[1]:off[2]]).decode() == s0
    with pytest.raises(IndexError):
        run([[] for _ in sub])


def test_assembly_emission_strands_random():
    """Emission strands on random hit tables (0-8 hits per read, garbage past each read's hit count, as
    the orientation kernel leaves it): equal to the running product of each read's hits, the column-wise
    form of the earlier build (per read, over all columns, masked)."""
    from types import SimpleNamespace

    rng = np.random.default_rng(5)
    for H in (4, 8):
        n_iso = 300
        m = rng.integers(1, 12, n_iso)
        sub_off = np.zeros(n_iso + 1, np.int64)
        np.cumsum(m, out=sub_off[1:])
        n_sub = int(sub_off[-1])
        nh = rng.integers(0, H + 1, n_sub).astype(np.int32)
        nh[sub_off[:-1]] = np.maximum(nh[sub_off[:-1]], 1)  # every isoform has an emission
        hits = rng.integers(-128, 128, (n_sub, H)).astype(np.int8)  # garbage ...
        valid = np.arange(H)[None, :] < nh[:, None]
        hits[valid] = np.where(rng.random(int(valid.sum())) < 0.5, 1, -1)  # ... except the hits
        res = SimpleNamespace(sub_off=sub_off, sub=np.arange(n_sub, dtype=np.int64),
                              seq_off=np.arange(n_sub, dtype=np.int64) * 10, seq_len=np.full(n_sub, 9, np.int32))
        a = define.Assembly(res, hits, nh)
        signs = np.cumprod(np.where(valid, hits, 1).astype(np.int64), axis=1)
        assert np.array_equal(a.e_read, np.repeat(np.arange(n_sub), nh))
        assert np.array_equal(a.e_sign, signs[valid].astype(np.int8))
        assert a.e_sign.dtype == np.int8


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, d, gtf_path, seed, q):
    from mandalorion_amd.comm import Comm

    comm = Comm(world, rank, "127.0.0.1", port)  # host transport (no device context)
    try:
        st = define.define_isoforms(d, cutoff=P["cutoff"], genome_file=gtf_path, splice_site_width=P["splice_site_width"],
                                    minimum_read_count=P["minimum_read_count"],
                                    white_list_polyA=P["white_list_polyA"].split(","), threads=2,
                                    junctions=P["junctions"], upstream_buffer=P["upstream_buffer"],
                                    downstream_buffer=P["downstream_buffer"], seed=seed, orient_fn=_stub_orient,
                                    consensus_fn=lambda s, o, g, sd: _first_of_groups(s, o, g), comm=comm,
                                    cluster_fn=ocl.cluster_loci)
        q.put((rank, st["loci"], st["isoforms"], comm.backend))
    finally:
        comm.close()


def test_sharded_two_ranks_host_comm(dataset, tmp_path):
    """Loci sharded over 2 ranks (LPT on file size), gathered on rank 0: output identical to 1 rank."""
    import multiprocessing as mp

    d, roots, info = dataset
    exp = GOLD["seeds"]["7"]
    for f in ("Isoform_Consensi.fasta", "reads2isoforms.txt"):
        p = os.path.join(d, f)
        if os.path.exists(p):
            os.remove(p)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_rank_main, args=(r, 2, port, d, info["gtf"], 7, q)) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(120)
        assert p.exitcode == 0
    got = sorted(q.get() for _ in range(2))
    assert got[0][3] == got[1][3] == "host"
    assert got[0][2] + got[1][2] == len(exp["isoform_headers"])  # isoforms split across ranks
    assert got[0][2] > 0 and got[1][2] > 0
    sha = lambda f: hashlib.sha256(open(os.path.join(d, f), "rb").read()).hexdigest()
    assert sha("Isoform_Consensi.fasta") == exp["isoform_consensi_sha256"]
    assert sha("reads2isoforms.txt") == exp["reads2isoforms_sha256"]


def test_bounds_index_equals_locus_bounds(dataset):
    """gtf.BoundsIndex (sorted lists + binary search) == the per-locus scan of the reference's bounds
    (defineIsoforms.py:140-150), up to list order, which make_genome_bins sorts away."""
    d, roots, info = dataset
    _, lb, rb, _ = gtf.parse_genome(info["gtf"], P["white_list_polyA"].split(","))
    bi = gtf.BoundsIndex(lb, rb)
    assert bi
    for r in roots + ["chrNone~1~100"]:
        c, a, b = r.split("~")
        want = gtf.locus_bounds(lb, rb, c, int(a), int(b))
        got = bi.bounds(c, int(a), int(b))
        assert [sorted(x) for x in want] == [x.tolist() for x in got]
    assert not gtf.BoundsIndex({}, {})
