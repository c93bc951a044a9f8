"""The D module against the UNMODIFIED reference run end to end with real consensi and orientation
(tests/golden/define_vectors.json, made by tests/golden/make_define_vectors.py): 35-40 % '-' strand
records, >100-read isoforms (subsample cap), 8-11 kb loci that take abPOA's `-S` branch.

* CPU (not gpu): the driver with the oracle's clustering, orientation and POA injected must write the reference's
  exact Isoform_Consensi.fasta / reads2isoforms.txt — pins rebinding, revcomp, fallbacks, `-S`
  selection and the writer against the reference's own code.
* GPU: the product path (HIP clustering + HIP orientation + HIP POA) must write the same bytes.
"""
from __future__ import annotations

import hashlib
import json
import os

import pytest

from mandalorion_amd import define, synth
from oracle import cluster as ocl

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "define_vectors.json")))
P = GOLD["params"]


def sha(path):
    return hashlib.sha256(open(path, "rb").read()).hexdigest()


def _dataset(tmp_path, name):
    spec = dict(GOLD["datasets"][name]["synth"])
    n = spec.pop("n_loci")
    d = str(tmp_path / name)
    recs = synth.write_loci(os.path.join(d, "tmp_SS"), n, threads=4, **spec)
    inp = GOLD["datasets"][name]["inputs"]
    assert recs == inp["records"]
    got = {f: sha(os.path.join(d, "tmp_SS", f)) for f in sorted(os.listdir(os.path.join(d, "tmp_SS")))}
    assert got == inp["psl_sha256"], "synthetic input differs from the one the reference ran on"
    return d


def _run(d, **kw):
    return define.define_isoforms(d, cutoff=P["cutoff"], genome_file="None", splice_site_width=P["splice_site_width"],
                                  minimum_read_count=P["minimum_read_count"],
                                  white_list_polyA=P["white_list_polyA"].split(","), threads=8,
                                  junctions=P["junctions"], upstream_buffer=P["upstream_buffer"],
                                  downstream_buffer=P["downstream_buffer"], seed=GOLD["seed"], **kw)


def _check(d, name, st):
    ref = GOLD["datasets"][name]["reference"]
    headers = [l[1:].rstrip("\n") for l in open(os.path.join(d, "Isoform_Consensi.fasta")) if l.startswith(">")]
    assert headers == ref["isoform_headers"]
    assert sha(os.path.join(d, "reads2isoforms.txt")) == ref["reads2isoforms_sha256"]
    assert sha(os.path.join(d, "Isoform_Consensi.fasta")) == ref["isoform_consensi_sha256"]
    assert st["poa_groups"] == ref["n_abpoa_calls"]


@pytest.mark.parametrize("name", sorted(GOLD["datasets"]))
def test_driver_with_oracle_equals_reference(tmp_path, name):
    from oracle import orient as oref
    from oracle import poa as opoa

    d = _dataset(tmp_path, name)
    seeded = []

    def cons(s, o, g, sd):
        seeded.append(int(sd.sum()) if sd is not None else 0)
        return opoa.consensus_packed(s, o, g, seeding=sd)

    st = _run(d, orient_fn=lambda s, o, g: oref.orient_packed(s, o, g), consensus_fn=cons, cluster_fn=ocl.cluster_loci)
    _check(d, name, st)
    assert sum(seeded) == GOLD["datasets"][name]["reference"]["n_seeded_calls"]


@pytest.mark.parametrize("name", ["config1", "r2c2_rev"])
def test_driver_uneven_chunks_equals_reference(tmp_path, name):
    """A three-chunk plan with uneven cuts (0.2 / 0.7 of the bytes: each chunk's part of both files
    streamed out as its POA finishes) writes the reference's exact files."""
    from oracle import orient as oref
    from oracle import poa as opoa

    d = _dataset(tmp_path, name)
    st = _run(d, orient_fn=lambda s, o, g: oref.orient_packed(s, o, g),
              consensus_fn=lambda s, o, g, sd: opoa.consensus_packed(s, o, g, seeding=sd), cluster_fn=ocl.cluster_loci,
              chunk_fracs=[0.2, 0.7])
    assert st["chunks"] == 3
    _check(d, name, st)


def test_driver_rank_shares_partition_the_loci(tmp_path):
    """share=(r, N) runs rank r's loci of the N-rank LPT plan alone (bench.py --share): the shares of a
    2-rank plan together hold every record and isoform of the one-rank run, each exactly once."""
    from oracle import orient as oref
    from oracle import poa as opoa

    d = _dataset(tmp_path, "config1")
    kw = dict(orient_fn=lambda s, o, g: oref.orient_packed(s, o, g),
              consensus_fn=lambda s, o, g, sd: opoa.consensus_packed(s, o, g, seeding=sd), cluster_fn=ocl.cluster_loci)
    full = _run(d, **kw)
    names = lambda: sorted(l.split("\t")[0] for l in open(os.path.join(d, "reads2isoforms.txt")))
    all_reads = names()
    got, reads = [], []
    for r in range(2):
        st = _run(d, share=(r, 2), **kw)
        got.append((st["records"], st["isoforms"]))
        reads += names()
    assert sum(x[0] for x in got) == full["records"] and sum(x[1] for x in got) == full["isoforms"]
    assert all(x[0] > 0 for x in got) and sorted(reads) == all_reads


def test_driver_three_rank_reassembly_in_one_process(tmp_path, monkeypatch):
    """The 3-rank gather reassembly (MANDO_REASSEMBLY=gather) with the transport replaced by an in-process
    hand-over: ranks 1 and 2 run their shares and hand their compacted payloads over, rank 0 runs its
    share, receives them and writes files byte-identical to the reference's."""
    import numpy as np
    from oracle import orient as oref
    from oracle import poa as opoa

    monkeypatch.setattr(define, "_REASSEMBLY", "gather")
    store = {}

    class Rec:
        def __init__(self, rank):
            self.rank, self.world = rank, 3

        def gather_bytes(self, blob):
            store[self.rank] = np.array(blob, copy=True)
            if self.rank:
                return None, None
            parts = [store[r] for r in range(3)]
            return np.concatenate(parts), np.array([p.size for p in parts])

    d = _dataset(tmp_path, "r2c2_rev")
    kw = dict(orient_fn=lambda s, o, g: oref.orient_packed(s, o, g),
              consensus_fn=lambda s, o, g, sd: opoa.consensus_packed(s, o, g, seeding=sd), cluster_fn=ocl.cluster_loci)
    groups = 0
    for r in (1, 2, 0):
        st = _run(d, comm=Rec(r), **kw)
        assert st["reassembly"] == "gather"
        groups += st["poa_groups"]
    st["poa_groups"] = groups  # each rank counts its own POA calls
    _check(d, name="r2c2_rev", st=st)


class PlaceRehearsal:
    """In-process stand-in for a communicator under placement reassembly: call c of allgather_bytes
    returns every rank's latest contribution to call c (ranks that have not made it yet: an empty one).
    Ranks run one after another, so an exchange whose inputs depend on k earlier exchanges is complete
    in pass k + 2: the counts in the second pass, the sizes computed from them in the third, the range
    placement's pieces (sent to the ranks that own their bytes of each file) in the fourth
    (tools/rank_rehearsal.py uses the same scheme)."""

    def __init__(self, rank, world, store):
        self.rank, self.world, self.store, self.calls = rank, world, store, 0

    def allgather_bytes(self, blob):
        import numpy as np

        c = self.store.setdefault(self.calls, {})
        self.calls += 1
        c[self.rank] = np.array(blob, dtype=np.uint8, copy=True)
        empty = np.zeros(1, np.int64).view(np.uint8)
        parts = [c.get(r, empty) for r in range(self.world)]
        return np.concatenate(parts), np.array([p.size for p in parts], dtype=np.int64)

    def barrier(self):
        pass


def test_driver_three_rank_placement_in_one_process(tmp_path):
    """The 3-rank placement reassembly (the default): the ranks exchange per-root isoform counts and byte
    sizes and each writes its own roots' blocks of both files; the files are the reference's bytes."""
    from oracle import orient as oref
    from oracle import poa as opoa

    d = _dataset(tmp_path, "r2c2_rev")
    kw = dict(orient_fn=lambda s, o, g: oref.orient_packed(s, o, g),
              consensus_fn=lambda s, o, g, sd: opoa.consensus_packed(s, o, g, seeding=sd), cluster_fn=ocl.cluster_loci)
    store = {}
    for _ in range(4):
        groups = 0
        for r in range(3):
            st = _run(d, comm=PlaceRehearsal(r, 3, store), **kw)
            assert st["reassembly"] == "place"
            groups += st["poa_groups"]
    st["poa_groups"] = groups
    _check(d, name="r2c2_rev", st=st)


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(GOLD["datasets"]))
def test_gpu_driver_equals_reference(gpu_ctx, tmp_path, name):
    d = _dataset(tmp_path, name)
    st = _run(d)
    _check(d, name, st)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["config1", "r2c2_rev", "long_seeded"])
def test_gpu_driver_sub_batched_clustering_equals_reference(gpu_ctx, tmp_path, monkeypatch, name):
    """Clustering in 3 sub-batches overlapped with the reading and copy (the large-input path, forced by
    MANDO_CL_SUB): the reference's files."""
    monkeypatch.setenv("MANDO_CL_SUB", "3")
    d = _dataset(tmp_path, name)
    st = _run(d)
    _check(d, name, st)


# ---------------------------------------------------------------------------------------------
# sharded runs: loci LPT-sharded over 2 ranks, one all-gather to rank 0's writer
# ---------------------------------------------------------------------------------------------
def _free_port():
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _shard_rank(rank, world, port, d, use_oracle, q, rccl=False):
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from mandalorion_amd.comm import Comm

    if rccl:  # one GPU per rank, RCCL reassembly (the product's multi-GPU path)
        os.environ.update(WORLD_SIZE=str(world), RANK=str(rank), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                          MASTER_PORT=str(port))
        c = Comm.from_env(device=rank)
        try:
            st = _run(d, comm=c, device=rank)
            q.put((rank, st["isoforms"], c.backend))
        finally:
            c.close()
        return

    kw = {}
    if use_oracle:
        from oracle import orient as oref
        from oracle import poa as opoa

        kw = dict(orient_fn=lambda s, o, g: oref.orient_packed(s, o, g),
                  consensus_fn=lambda s, o, g, sd: opoa.consensus_packed(s, o, g, seeding=sd),
                  cluster_fn=ocl.cluster_loci)
    with Comm(world, rank, "127.0.0.1", port, timeout_s=120) as c:  # host transport (one GPU or none)
        st = _run(d, comm=c, **kw)
        q.put((rank, st["isoforms"], c.backend))


def _sharded(d, use_oracle, world=2, rccl=False):
    import multiprocessing as mp

    for f in ("Isoform_Consensi.fasta", "reads2isoforms.txt"):
        if os.path.exists(os.path.join(d, f)):
            os.remove(os.path.join(d, f))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_shard_rank, args=(r, world, port, d, use_oracle, q, rccl)) for r in range(world)]
    for p in ps:
        p.start()
    got = sorted(q.get(timeout=300) for _ in range(world))
    for p in ps:
        p.join(120)
        assert p.exitcode == 0
    assert all(g[1] > 0 for g in got)  # every rank got loci
    return got


@pytest.mark.parametrize("world,mode", [(2, "place"), (3, "place"), (2, "gather")])
def test_sharded_ranks_equal_reference(tmp_path, monkeypatch, world, mode):
    """world rank processes over the host transport, placement (the default) or gather reassembly: the
    reference's files."""
    d = _dataset(tmp_path, "r2c2_rev")
    monkeypatch.setenv("MANDO_REASSEMBLY", mode)
    _sharded(d, use_oracle=True, world=world)
    ref = GOLD["datasets"]["r2c2_rev"]["reference"]
    assert sha(os.path.join(d, "reads2isoforms.txt")) == ref["reads2isoforms_sha256"]
    assert sha(os.path.join(d, "Isoform_Consensi.fasta")) == ref["isoform_consensi_sha256"]


# BASELINE configs[3] shape (10M mixed R2C2 + PacBio 2-4 kb, sharded): a small slice of it
CONFIG4_SLICE = dict(reads=(40, 60), exons=(5, 12), exon_len=(130, 570), pacbio_frac=0.2, rev_frac=0.5, seed=4)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["config1", "sirv_like"])
def test_gpu_driver_two_chunks_equals_reference(gpu_ctx, tmp_path, name):
    """The product path in two pipelined chunks (the second clustered and oriented while the first one's
    POA runs): two POA launches, the reference's files."""
    d = _dataset(tmp_path, name)
    st = _run(d, n_chunks=2)
    assert st["chunks"] == 2 and len(st["poa_launches"]) == 2
    _check(d, name, st)


@pytest.mark.gpu
@pytest.mark.parametrize("world,mode", [(2, "place"), (3, "place"), (2, "gather")])
def test_gpu_config4_slice_sharded_equals_one_rank(gpu_ctx, tmp_path, monkeypatch, world, mode):
    """world rank processes on the one GPU (host transport), each placing its blocks into the shared
    files at once (or gathering to rank 0): byte-identical to the one-rank files."""
    d = str(tmp_path / "c4")
    synth.write_loci(os.path.join(d, "tmp_SS"), 96, threads=8, **CONFIG4_SLICE)
    _run(d)
    one = [open(os.path.join(d, f), "rb").read() for f in ("Isoform_Consensi.fasta", "reads2isoforms.txt")]
    monkeypatch.setenv("MANDO_REASSEMBLY", mode)  # read by the spawned ranks' define module
    _sharded(d, use_oracle=False, world=world)
    two = [open(os.path.join(d, f), "rb").read() for f in ("Isoform_Consensi.fasta", "reads2isoforms.txt")]
    assert one == two
    if world > 2 or mode != "place":
        return
    # and the one-rank GPU files equal the CPU restatements' on the same slice
    from oracle import orient as oref
    from oracle import poa as opoa

    _run(d, orient_fn=lambda s, o, g: oref.orient_packed(s, o, g),
         consensus_fn=lambda s, o, g, sd: opoa.consensus_packed(s, o, g, seeding=sd), cluster_fn=ocl.cluster_loci)
    assert [open(os.path.join(d, f), "rb").read() for f in ("Isoform_Consensi.fasta", "reads2isoforms.txt")] == one


@pytest.mark.gpu
def test_gpu_config4_slice_two_gpus_rccl_equals_one_rank(gpu_ctx, tmp_path):
    """Two ranks on two GPUs with the RCCL all-gather: byte-identical to the one-rank files.  Needs two
    visible GPUs; skipped on a one-GPU box."""
    from mandalorion_amd import _lib

    if _lib.device_count() < 2:
        pytest.skip("two GPUs needed for two RCCL ranks")
    d = str(tmp_path / "c4")
    synth.write_loci(os.path.join(d, "tmp_SS"), 96, threads=8, **CONFIG4_SLICE)
    _run(d)
    one = [open(os.path.join(d, f), "rb").read() for f in ("Isoform_Consensi.fasta", "reads2isoforms.txt")]
    got = _sharded(d, use_oracle=False, rccl=True)
    assert all(g[2] == "rccl" for g in got)
    two = [open(os.path.join(d, f), "rb").read() for f in ("Isoform_Consensi.fasta", "reads2isoforms.txt")]
    assert one == two
