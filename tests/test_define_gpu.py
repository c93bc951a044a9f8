"""End-to-end D module on the GPU: clustering (HIP) -> orientation (HIP) -> batched POA (HIP) ->
writer, against the same driver with the CPU restatements (oracle/) injected for orientation and POA.
The written Isoform_Consensi.fasta / reads2isoforms.txt must be byte-identical; reads2isoforms.txt must
also equal the reference's own (tests/golden/cluster_vectors.json, independent of consensus)."""
from __future__ import annotations

import hashlib
import json
import os

import pytest

from mandalorion_amd import define, simdata

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "cluster_vectors.json")))
P = GOLD["params"]


def _run(d, gtf, **kw):
    return define.define_isoforms(d, cutoff=P["cutoff"], genome_file=gtf, splice_site_width=P["splice_site_width"],
                                  minimum_read_count=P["minimum_read_count"],
                                  white_list_polyA=P["white_list_polyA"].split(","), threads=8,
                                  junctions=P["junctions"], upstream_buffer=P["upstream_buffer"],
                                  downstream_buffer=P["downstream_buffer"], seed=0, **kw)


@pytest.mark.gpu
def test_define_gpu_equals_cpu_restatement(gpu_ctx, tmp_path):
    from oracle import orient as oref
    from oracle import poa as opoa

    d = str(tmp_path)
    loci = simdata.make_dataset(simdata.fixture_specs())
    info = simdata.write_dataset(loci, d)
    st = _run(d, info["gtf"])
    read = lambda f: open(os.path.join(d, f), "rb").read()
    gpu_fa, gpu_r2i = read("Isoform_Consensi.fasta"), read("reads2isoforms.txt")
    assert hashlib.sha256(gpu_r2i).hexdigest() == GOLD["seeds"]["0"]["reads2isoforms_sha256"]
    assert st["poa_groups"] > 20
    from oracle import cluster as ocl

    _run(d, info["gtf"], orient_fn=lambda s, o, g: oref.orient_packed(s, o, g),
         consensus_fn=lambda s, o, g, sd: opoa.consensus_packed(s, o, g, seeding=sd), cluster_fn=ocl.cluster_loci)
    assert read("Isoform_Consensi.fasta") == gpu_fa
    assert read("reads2isoforms.txt") == gpu_r2i


@pytest.mark.gpu
def test_define_gpu_chunked_pipeline(gpu_ctx, tmp_path):
    """Three chunks: two POA launches in flight on two device contexts (slots 0 and 3) while the next
    chunk is oriented (slot 1); the files must equal the one-chunk run's."""
    d = str(tmp_path)
    loci = simdata.make_dataset(simdata.fixture_specs())
    info = simdata.write_dataset(loci, d)
    read = lambda f: open(os.path.join(d, f), "rb").read()
    _run(d, info["gtf"])
    one = read("Isoform_Consensi.fasta"), read("reads2isoforms.txt")
    st = _run(d, info["gtf"], n_chunks=3)
    assert st["chunks"] == 3 and len(st["poa_launches"]) == 3
    assert (read("Isoform_Consensi.fasta"), read("reads2isoforms.txt")) == one


@pytest.mark.gpu
def test_define_gpu_byte_capped_chunks_then_one_chunk(gpu_ctx, tmp_path, monkeypatch):
    """The byte-capped many-chunk branch (config 4's plan, thresholds lowered to this small input), then a
    one-chunk call in the same process: same files each time, and the one-chunk call's POA workspaces are
    sized exactly as before the many-chunk call (its budget comes from its own plan; nothing of the
    many-chunk plan survives in the process)."""
    from mandalorion_amd import _lib

    d = str(tmp_path)
    loci = simdata.make_dataset(simdata.fixture_specs())
    info = simdata.write_dataset(loci, d)
    read = lambda f: open(os.path.join(d, f), "rb").read()
    pctx = _lib.context(0, 0)
    env0 = dict(os.environ)
    _run(d, info["gtf"])
    one = read("Isoform_Consensi.fasta"), read("reads2isoforms.txt")
    slots1 = pctx.last_slots()
    text = sum(os.path.getsize(os.path.join(d, "tmp_SS", f)) for f in os.listdir(os.path.join(d, "tmp_SS")))
    with monkeypatch.context() as m:
        m.setattr(define, "_TWO_CHUNK_BYTES", 1)
        m.setattr(define, "_MIN_LOCI_CHUNKED", 1)
        m.setattr(define, "_CHUNK_BYTES", text // 3 + 1)
        st = _run(d, info["gtf"])
        assert st["chunks"] >= 4 and len(st["poa_launches"]) >= 3
        assert (read("Isoform_Consensi.fasta"), read("reads2isoforms.txt")) == one
        # the many-chunk call's launches were sized from its own (smaller) budget
        assert sum(pctx.last_slots()[1]) <= sum(slots1[1])
    assert dict(os.environ) == env0
    _run(d, info["gtf"])
    assert (read("Isoform_Consensi.fasta"), read("reads2isoforms.txt")) == one
    assert pctx.last_slots() == slots1


@pytest.mark.gpu
def test_define_gpu_hbm_plan_after_a_larger_call(gpu_ctx, tmp_path):
    """A whole-input call, then a rank-share call (a smaller plan) in the same process -- the round-4
    rehearsal's sequence, whose second call ran out of HBM: the clustering caches the larger call left
    are trimmed to the second call's plan, so what they hold plus the POA grant stays within the usable
    HBM, the POA workspaces stay within their grant, and the share's files hold its own loci."""
    from mandalorion_amd import _lib

    d = str(tmp_path)
    loci = simdata.make_dataset(simdata.fixture_specs())
    info = simdata.write_dataset(loci, d)
    st1 = _run(d, info["gtf"])
    st2 = _run(d, info["gtf"], share=(0, 4))
    for st in (st1, st2):
        h = st["hbm"]
        assert h["cache_held_start"] + h["poa_budget"] <= define._HBM_USABLE * h["total"]
        assert h["poa_ws_held"] <= h["poa_budget"]
    # the share's caches were trimmed to its (smaller) largest chunk before its POA grant was sized
    assert st2["hbm"]["cache_held_start"] <= st1["hbm"]["cache_held_end"]
    assert 0 < st2["records"] < st1["records"]
    # the budget is the call's own: back to the library's default policy afterwards
    pctx = _lib.context(0, 0)
    free0, total = _lib.device_memory(0)
    assert 0 < free0 <= total
    assert pctx.memory()[1] <= st1["hbm"]["poa_budget"]


@pytest.mark.gpu
def test_gpu_config3_clustering_equals_reference_run(gpu_ctx, tmp_path):
    """BASELINE configs[2] at full size (20,000 loci, 1M records): the GPU run's reads2isoforms.txt and
    isoform header list equal the UNMODIFIED reference's own run on the same data
    (tests/golden/make_reference_fullsize.py: defineIsoforms.py under a seeded parent, 70 min of its Python
    here), and both files equal the oracle's full-size hashes (bench.fullsize_check)."""
    import bench

    wl = bench.WORKLOADS["config3"]
    d = str(tmp_path / "c3")
    bench.gen_data(d, wl, wl["loci"], 16)
    define.define_isoforms(d, threads=16, device=0)
    ok, scope = bench.fullsize_check(d, f"config3:{wl['loci']}")
    assert ok and scope == f"all {wl['loci']} loci"
