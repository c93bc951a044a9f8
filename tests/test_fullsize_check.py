"""bench.fullsize_check's comparison of a run's files with the oracle's full-size hashes and with the
reference's own run (whole files, or a sorted-root prefix of them): host logic on small files, no GPU."""
from __future__ import annotations

import hashlib
import json
import os

import pytest

import bench


def _sha(b: bytes) -> str:
    return hashlib.sha256(b).hexdigest()


def _heads(fa: bytes, k: int) -> str:
    lines = [l + b"\n" for l in fa.split(b"\n") if l.startswith(b">")]
    return _sha(b"".join(lines[:k]))


def test_fullsize_check_oracle_and_reference(tmp_path, monkeypatch):
    d = str(tmp_path)
    fa = b"".join(b">Isoform%d_2\nACGT\n" % k for k in range(1, 11))
    r2 = b"".join(b"r%da\tIsoform%d_2\nr%db\tIsoform%d_2\n" % (k, k, k, k) for k in range(1, 11))
    open(os.path.join(d, "Isoform_Consensi.fasta"), "wb").write(fa)
    open(os.path.join(d, "reads2isoforms.txt"), "wb").write(r2)
    ent = {"isoform_consensi_sha256": _sha(fa), "reads2isoforms_sha256": _sha(r2), "loci": 10}
    # the reference run on the first loci: the first 4 isoforms' lines of both files
    p_r2 = b"".join(l + b"\n" for l in r2.split(b"\n")[:8])
    ent["reference_prefix"] = {"loci": 4, "isoforms": 4, "reads2isoforms_bytes": len(p_r2),
                               "reads2isoforms_sha256": _sha(p_r2), "headers_sha256": _heads(fa, 4)}
    hashes = tmp_path / "h.json"
    hashes.write_text(json.dumps({"w:10": ent}))
    monkeypatch.setattr(bench, "FULLSIZE_HASHES", str(hashes))
    assert bench.fullsize_check(d, "w:10") == (True, "first 4 of 10 loci (sorted roots)")
    assert bench.fullsize_check(d, "other:1") == (None, None)
    # the whole-file form
    ent.pop("reference_prefix")
    ent.update(reference_reads2isoforms_sha256=_sha(r2), reference_headers_sha256=_heads(fa, 10))
    hashes.write_text(json.dumps({"w:10": ent}))
    assert bench.fullsize_check(d, "w:10") == (True, "all 10 loci")
    # a clustering difference fails the run
    ent["reference_headers_sha256"] = "0" * 64
    hashes.write_text(json.dumps({"w:10": ent}))
    with pytest.raises(SystemExit):
        bench.fullsize_check(d, "w:10")
