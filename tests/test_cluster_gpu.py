"""HIP clustering kernels (csrc/cluster_kernel.hip) against the clustering restatement
(oracle/cluster_ref.cpp, itself pinned to the reference by tests/golden/*_vectors.json), locus by locus:
status, peaks (with the rounded proportion), isoform members in IsoDict order, the subsample in draw
order, and the records' name / sequence spans.  Data: the reference-pinned datasets, a config-3-shaped
sample, config-4 / config-5 shapes, and hand-made edge cases (malformed lines, bad strands, CRLF,
missing trailing newline, accuracies around 0.9, other chromosomes, empty files).
"""
from __future__ import annotations

import json
import os

import numpy as np
import pytest

from mandalorion_amd import cluster, define, gtf, simdata, synth
from oracle import cluster as ocl

pytestmark = pytest.mark.gpu

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "define_vectors.json")))


def _inputs(d, ann_gtf=None):
    tmp = os.path.join(d, "tmp_SS")
    roots = define._roots(tmp)
    paths = [os.path.join(tmp, r + ".psl") for r in roots]
    chroms = [r.split("~")[0] for r in roots]
    ann = None
    if ann_gtf:
        _, lb, rb, _ = gtf.parse_genome(ann_gtf, ["0"])
        ann = [gtf.locus_bounds(lb, rb, r.split("~")[0], int(r.split("~")[1]), int(r.split("~")[2])) for r in roots]
    return roots, paths, chroms, ann


def _compare(paths, chroms, ann=None, **kw):
    want = ocl.cluster_loci(paths, chroms, ann=ann, threads=8, **kw)
    got = cluster.cluster_loci(paths, chroms, ann=ann, threads=8, **kw)
    try:
        assert got.n_loci == want.n_loci
        bad = np.nonzero(got.locus_status != want.locus_status)[0]
        assert len(bad) == 0, f"locus {paths[bad[0]]}: status {got.locus_status[bad[0]]} vs {want.locus_status[bad[0]]}"
        ok = want.locus_status == 0
        # records of ok loci: same spans
        rl = want.rec_locus
        sel = ok[rl] if len(rl) else np.zeros(0, bool)
        grl = got.rec_locus
        gsel = ok[grl] if len(grl) else np.zeros(0, bool)
        for f in ("name_off", "name_len", "seq_off", "seq_len", "rec_locus"):
            a, b = getattr(got, f)[gsel], getattr(want, f)[sel]
            if not np.array_equal(a, b):
                i = int(np.nonzero(a != b)[0][0]) if len(a) == len(b) else -1
                raise AssertionError(f"{f} differs (first at {i})")
        for li in np.nonzero(ok)[0]:
            gp = [(p.start, p.end, p.type, p.side, p.prop_str) for p in got.peaks(int(li))]
            wp = [(p.start, p.end, p.type, p.side, p.prop_str) for p in want.peaks(int(li))]
            assert gp == wp, f"locus {paths[li]}: peaks\n gpu {gp}\n ref {wp}"
        assert np.array_equal(got.iso_locus, want.iso_locus), "isoform count per locus differs"
        # members as locus-local record indices (a failed locus may hold a partial record list in the
        # restatement and none in the kernel's output, which shifts the global indices after it)
        g0 = np.searchsorted(got.rec_locus, np.arange(got.n_loci))
        w0 = np.searchsorted(want.rec_locus, np.arange(want.n_loci))
        for i in range(want.n_isoforms):
            li = int(want.iso_locus[i])
            a, b = got.members(i) - g0[li], want.members(i) - w0[li]
            assert np.array_equal(a, b), f"isoform {i} (locus {paths[li]}): members differ"
            a, b = got.subsample(i) - g0[li], want.subsample(i) - w0[li]
            assert np.array_equal(a, b), f"isoform {i} (locus {paths[li]}): subsample differs"
        return int(ok.sum()), want.n_isoforms
    finally:
        got.close()
        want.close()


def test_fixture_loci_with_annotation(tmp_path):
    d = str(tmp_path)
    loci = simdata.make_dataset(simdata.fixture_specs())
    info = simdata.write_dataset(loci, d)
    roots, paths, chroms, ann = _inputs(d, info["gtf"])
    for seed in (0, 7):
        n_ok, n_iso = _compare(paths, chroms, ann=ann, seed=seed)
        assert n_ok == len(roots) and n_iso > 20
    _compare(paths, chroms, ann=None, seed=3)


@pytest.mark.parametrize("name", sorted(GOLD["datasets"]))
def test_reference_pinned_datasets(tmp_path, name):
    spec = dict(GOLD["datasets"][name]["synth"])
    n = spec.pop("n_loci")
    d = str(tmp_path)
    synth.write_loci(os.path.join(d, "tmp_SS"), n, threads=8, **spec)
    _, paths, chroms, _ = _inputs(d)
    n_ok, _ = _compare(paths, chroms)
    assert n_ok == n


@pytest.mark.parametrize("shape", ["config3", "config4", "config5"])
def test_bench_shapes(tmp_path, shape):
    kw = {"config3": dict(n=600, reads=(50, 50), exon_len=(200, 500), rev_frac=0.3),
          "config4": dict(n=600, reads=(40, 60), exon_len=(130, 570), pacbio_frac=0.2, rev_frac=0.5),
          "config5": dict(n=12, reads=(200, 200), exons=(8, 10), exon_len=(850, 1000), isoforms=(1, 1))}[shape]
    n = kw.pop("n")
    d = str(tmp_path)
    synth.write_loci(os.path.join(d, "tmp_SS"), n, threads=8, seed=11, **kw)
    _, paths, chroms, _ = _inputs(d)
    n_ok, _ = _compare(paths, chroms, seed=5)
    assert n_ok == n
    # non-default parameters: wider splice window, other buffers, min count 3, larger subsample
    _compare(paths[:100], chroms[:100], seed=1, splice_site_width=3, upstream_buffer=20, downstream_buffer=30,
             minimum_read_count=3, poa_subsample=150, cutoff=0.25, junctions="gtag,gcag")


@pytest.mark.parametrize("sub", ["3", "5"])
def test_sub_batched_calls_equal_the_restatement(tmp_path, monkeypatch, sub):
    """MANDO_CL_SUB: the loci clustered in byte-balanced sub-batches, each as soon as its text is on the
    device (copy stream + event), the rest still being read: the restatement's results, locus by locus
    (the default sub-batches only large calls: >= 1024 loci and 256 MB of text)."""
    d = str(tmp_path)
    synth.write_loci(os.path.join(d, "tmp_SS"), 300, threads=8, seed=17, reads=(40, 60), exon_len=(130, 570),
                     pacbio_frac=0.2, rev_frac=0.5)
    _, paths, chroms, _ = _inputs(d)
    monkeypatch.setenv("MANDO_CL_SUB", sub)
    n_ok, _ = _compare(paths, chroms, seed=5)
    assert n_ok == 300


def test_mixed_large_and_small_loci(tmp_path):
    """Loci of >= 2,048 records run on the several-wave kernel (helper waves join wave 0 for the coverage
    sets and the coverage merge), the others on one wave each, in the same call: both launches (and the
    order split between them) equal the restatement locus by locus."""
    d = str(tmp_path)
    synth.write_loci(os.path.join(d, "big", "tmp_SS"), 3, reads=(2100, 2600), exons=(6, 10), exon_len=(60, 200),
                     isoforms=(4, 8), threads=8, seed=31, rev_frac=0.3)
    synth.write_loci(os.path.join(d, "small", "tmp_SS"), 40, reads=(10, 60), threads=8, seed=32, rev_frac=0.3)
    # one-wave loci whose permutations, sorts and histogram bins outgrow the one-wave kernel's LDS
    # (global-memory permutation, sort passes and bins)
    synth.write_loci(os.path.join(d, "mid", "tmp_SS"), 3, reads=(1100, 1900), exons=(6, 10), exon_len=(60, 200),
                     isoforms=(4, 8), threads=8, seed=33, rev_frac=0.3)
    _, pb, cb, _ = _inputs(os.path.join(d, "big"))
    _, ps, cs, _ = _inputs(os.path.join(d, "small"))
    _, pm, cm, _ = _inputs(os.path.join(d, "mid"))
    n_ok, _ = _compare(ps[:20] + pb + pm + ps[20:], cs[:20] + cb + cm + cs[20:], seed=4)
    assert n_ok == len(pb) + len(ps) + len(pm)


def _edit_lines(src, dst, fn):
    lines = open(src).read().split("\n")
    if lines and lines[-1] == "":
        lines = lines[:-1]
    out = fn(lines)
    open(dst, "w").write(out)


def test_edge_cases(tmp_path):
    """Malformed and unusual locus files: the kernel must report the restatement's status (or agree)."""
    d = str(tmp_path)
    synth.write_loci(os.path.join(d, "src"), 24, reads=(12, 30), threads=4, seed=21, rev_frac=0.3)
    src = sorted(os.listdir(os.path.join(d, "src")))
    tmp = os.path.join(d, "tmp_SS")
    os.makedirs(tmp)
    srcp = lambda k: os.path.join(d, "src", src[k])

    def f(k, name, fn):
        _edit_lines(srcp(k), os.path.join(tmp, name), fn)

    def col(lines, i, c, v):
        a = lines[i].split("\t")
        a[c] = v
        lines[i] = "\t".join(a)
        return lines

    f(0, "chrA~1~2.psl", lambda L: "\n".join(L))  # no trailing newline
    f(1, "chrA~3~4.psl", lambda L: "\r\n".join(L) + "\r\n")  # CRLF
    f(2, "chrA~5~6.psl", lambda L: "\n".join(col(L, 3, 8, "x")) + "\n")  # bad strand
    f(3, "chrA~7~8.psl", lambda L: "\n".join(L[:4] + ["a\tb\tc"] + L[4:]) + "\n")  # short line
    f(4, "chrA~9~10.psl", lambda L: "\n".join(L) + "\n\n")  # trailing empty line
    f(5, "chrA~11~12.psl", lambda L: "\n".join(col(L, 0, 10, "12x")) + "\n")  # bad int
    f(6, "chrA~13~14.psl", lambda L: "\n".join(col(col(col(L, 0, 21, "0.9"), 1, 21, "0.8999999999999999666"),
                                                   2, 21, "8.99999999999999966693309261245303787291049957275390626e-1")) + "\n")
    f(7, "chrA~15~16.psl", lambda L: "\n".join(col(col(L, 0, 21, "nan"), 1, 21, " 1e-05 ")) + "\n")
    f(8, "chrA~17~18.psl", lambda L: "\n".join(col(L, 2, 13, "chrOther")) + "\n")  # another chromosome
    f(9, "chrA~19~20.psl", lambda L: "\n".join([" " + L[0]] + L[1:]) + "\n")  # leading space
    f(10, "chrA~21~22.psl", lambda L: "\n".join(col(L, 1, 18, L[1].split("\t")[18] + "5,")) + "\n")  # block count mismatch
    f(11, "chrA~23~24.psl", lambda L: "\n".join(l + "\textra" for l in L) + "\n")  # a 25th column
    f(12, "chrA~25~26.psl", lambda L: "\n".join(col(L, 0, 22, L[0].split("\t")[22].replace("~", "~x", 1))) + "\n")  # bad cs intron
    f(13, "chrA~27~28.psl", lambda L: "\n".join(col(L, 0, 21, "abc")) + "\n")  # bad accuracy
    open(os.path.join(tmp, "chrA~29~30.psl"), "w").close()  # empty file
    f(14, "chrA~31~32.psl", lambda L: "\n".join(col(L, 4, 8, "-")) + "\n")
    f(15, "chrA~33~34.psl", lambda L: "\n".join(L[:1]) + "\n")  # one record
    roots = define._roots(tmp)
    paths = [os.path.join(tmp, r + ".psl") for r in roots]
    # the synthetic records are on chr<k>: pass each file's own chromosome (col 13 of its first line)
    chroms = []
    for p in paths:
        first = open(p).readline().split("\t")
        chroms.append(first[13] if len(first) > 13 else "chrA")
    _compare(paths, chroms, seed=2)
    _compare(paths + ["/nonexistent/x.psl"], chroms + ["chrA"], seed=2)


def test_large_files_on_several_waves(tmp_path):
    """Locus files of 4 MB or more are parsed by several waves (K1: line ends and records split between
    them): such files without a trailing newline, with CRLF ends, and with a malformed line in the middle
    (a parse error, wherever the split falls) equal the restatement."""
    d = str(tmp_path)
    synth.write_loci(os.path.join(d, "src"), 1, reads=(7000, 7000), exons=(10, 14), exon_len=(60, 200),
                     isoforms=(9, 11), threads=8, seed=41, rev_frac=0.3)
    src = os.path.join(d, "src", sorted(os.listdir(os.path.join(d, "src")))[0])
    assert os.path.getsize(src) >= 4 << 20
    tmp = os.path.join(d, "tmp_SS")
    os.makedirs(tmp)
    chrom = open(src).readline().split("\t")[13]
    _edit_lines(src, os.path.join(tmp, f"{chrom}~1~2.psl"), lambda L: "\n".join(L))  # no trailing newline
    _edit_lines(src, os.path.join(tmp, f"{chrom}~3~4.psl"), lambda L: "\r\n".join(L) + "\r\n")
    _edit_lines(src, os.path.join(tmp, f"{chrom}~5~6.psl"),
                lambda L: "\n".join(L[:4321] + ["a\tb\tc"] + L[4321:]) + "\n")  # short line
    roots = define._roots(tmp)
    paths = [os.path.join(tmp, r + ".psl") for r in roots]
    _compare(paths, [chrom] * len(paths), seed=6)


def test_repeated_calls_reuse_buffers(tmp_path):
    """Back-to-back calls reuse the host and device text buffers and the per-context scratch; every call
    must equal the restatement (a refilled, recycled buffer once handed the kernels stale bytes)."""
    spec = dict(GOLD["datasets"]["sirv_like"]["synth"])
    n = spec.pop("n_loci")
    d = str(tmp_path)
    synth.write_loci(os.path.join(d, "tmp_SS"), n, threads=8, **spec)
    _, paths, chroms, _ = _inputs(d)
    want = ocl.cluster_loci(paths, chroms, threads=8)
    ref = (want.locus_status.tolist(), want.mem.tolist(), want.sub.tolist())
    want.close()
    for _ in range(6):
        got = cluster.cluster_loci(paths, chroms, threads=8)
        assert (got.locus_status.tolist(), got.mem.tolist(), got.sub.tolist()) == ref
        got.close()
