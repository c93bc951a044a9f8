"""Gene grouping (mandalorion_amd/genes.py) against the reference's groupIsoforms.py output on the same
synthetic files (tests/golden/gene_vectors.json, made by tests/golden/make_gene_vectors.py)."""
import gzip
import json
import os

import pytest

from mandalorion_amd import genes

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "gene_vectors.json")))


def _run(tmp_path, annotation):
    p = tmp_path / "Isoforms.sorted.psl"
    p.write_text(GOLD["psl"])
    o = tmp_path / "genes.txt"
    genes.group_isoforms(str(p), str(o), annotation)
    out = []
    for line in o.read_text().splitlines():
        a = line.split("\t")
        out.append(a[:6] + [a[6].split(",") if a[6] else []])
    return out


def test_grouping_matches_reference_annotated(tmp_path):
    g = tmp_path / "ann.gtf"
    g.write_text(GOLD["gtf"])
    got = _run(tmp_path, str(g))
    assert len(got) == len(GOLD["annotated"])
    for a, b in zip(got, GOLD["annotated"]):
        assert a == b
    assert any(len(a[6]) > 1 for a in got)        # the fixture has loci with several genes


def test_grouping_matches_reference_gzip(tmp_path):
    g = tmp_path / "ann.gtf.gz"
    with gzip.open(g, "wt") as f:
        f.write(GOLD["gtf"])
    assert _run(tmp_path, str(g)) == GOLD["annotated"]


def test_grouping_matches_reference_unannotated(tmp_path):
    assert _run(tmp_path, "None") == GOLD["unannotated"]


def test_parity_counting_against_per_base_sets():
    """The interval counts equal a direct per-base count of the marked positions (groupIsoforms.py:72-83,
    :155-162) on random exons and blocks, both parities."""
    import numpy as np

    rng = np.random.default_rng(3)
    for _ in range(200):
        exons = [(int(s), int(s + rng.integers(1, 60))) for s in rng.integers(0, 300, size=rng.integers(1, 6))]
        blocks = [(int(s), int(s + rng.integers(1, 80))) for s in rng.integers(0, 300, size=rng.integers(1, 5))]
        marked = {i for s, e in exons for i in range(s, e, 2)}
        covered = {i for s, e in blocks for i in range(s, e)}
        cs, ce = genes._merge(blocks)
        es, ee = genes._merge([x for x in exons if x[0] % 2 == 0])
        os_, oe = genes._merge([x for x in exons if x[0] % 2 == 1])
        n = genes._count_parity(cs, ce, es, ee, False) + genes._count_parity(cs, ce, os_, oe, True)
        assert n == len(marked & covered)


def test_bad_annotation_suffix(tmp_path):
    p = tmp_path / "x.psl"
    p.write_text(GOLD["psl"])
    with pytest.raises(ValueError):
        genes.group_isoforms(str(p), str(tmp_path / "o"), str(tmp_path / "ann.txt"))
