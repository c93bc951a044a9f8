"""§8(f) row 1: PSL ingest + locus split (mando_split_loci) against the reference's own split
(GNU `sort -k 14,14 -k 16,17n` + get_chromosomes) on the same shuffled input: identical sorted file
and identical locus files (names and bytes).  Fixture: tests/golden/split_vectors.json."""
import hashlib
import importlib.util
import json
import os

from mandalorion_amd import psl

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = json.load(open(os.path.join(HERE, "golden", "split_vectors.json")))


def _make_input(path):
    spec = importlib.util.spec_from_file_location("msv", os.path.join(HERE, "golden", "make_split_vectors.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m.make_input(path)


def test_split_matches_reference(tmp_path):
    src = str(tmp_path / "clean.psl")
    assert _make_input(src) == GOLD["records"]
    srt = str(tmp_path / "clean.sorted.psl")
    nrec, nloc = psl.split_loci(src, str(tmp_path / "tmp_SS"), sort_lines=True, sorted_out=srt)
    assert nrec == GOLD["records"] and nloc == len(GOLD["loci"])
    assert hashlib.sha256(open(srt, "rb").read()).hexdigest() == GOLD["sorted_sha256"]
    got = {f: hashlib.sha256(open(tmp_path / "tmp_SS" / f, "rb").read()).hexdigest()
           for f in sorted(os.listdir(tmp_path / "tmp_SS"))}
    assert got == GOLD["loci"]


def test_split_presorted_input_is_idempotent(tmp_path):
    src = str(tmp_path / "clean.psl")
    _make_input(src)
    srt = str(tmp_path / "s1.psl")
    psl.split_loci(src, str(tmp_path / "a"), sort_lines=True, sorted_out=srt)
    psl.split_loci(srt, str(tmp_path / "b"), sort_lines=False)
    assert sorted(os.listdir(tmp_path / "a")) == sorted(os.listdir(tmp_path / "b"))


def test_mando_cli_P_then_D(tmp_path):
    """`Mando.py -M PD` on a clean PSL: split, then the D module (orientation / POA stand-ins are not
    injectable through the CLI, so only P and the D-module input checks run without a GPU)."""
    from mandalorion_amd import mando

    tmp = tmp_path / "tmp"
    tmp.mkdir()
    _make_input(str(tmp / "mm2Alignments.clean.psl"))
    fa = tmp_path / "reads.fasta"
    fa.write_text(">r\nACGT\n")
    assert mando.main(["-p", str(tmp_path), "-f", str(fa), "-M", "P"]) == 0
    assert sorted(os.listdir(tmp / "tmp_SS")) == sorted(GOLD["loci"])
    assert hashlib.sha256(open(tmp / "mm2Alignments.clean.sorted.psl", "rb").read()).hexdigest() == GOLD["sorted_sha256"]


def test_list_roots_matches_reference_scan(tmp_path):
    """mando_list_roots (native scan + stat + sort) == the reference's roots loop (defineIsoforms.py:130-139)
    restated in define._roots_py: sizes only for exact <root>.psl files, '.psl' cut at its first
    occurrence, directories skipped, symlinks followed, (chrom, int(start)) order."""
    import random

    from mandalorion_amd import define

    d = tmp_path / "tmp_SS"
    d.mkdir()
    rng = random.Random(5)
    for i in range(3000):
        c = rng.choice(["chr1", "chr10", "chr2", "chrX", "chrUn_KI270742v1", "é_chr"])
        s = rng.randrange(0, 10 ** 9)
        (d / f"{c}~{s}~{s + rng.randrange(1, 10 ** 5)}.psl").write_bytes(b"x" * rng.randrange(0, 50))
    (d / "chr1~5~9.psl.bak").write_bytes(b"ab")
    (d / "chr1~7~9.pslx").write_bytes(b"")
    (d / "dir.psl").mkdir()
    (d / "chr9~1~2.psl").symlink_to(d / "chr1~7~9.pslx")
    s1, s2 = {}, {}
    assert define._roots(str(d), s1) == define._roots_py(str(d), s2)
    assert s1 == s2
    # the multi-rank scan: names from one directory read, sizes stat'ed per slice
    names = define._root_names(str(d))
    assert names == define._roots_py(str(d))
    assert define._root_sizes(str(d), names).tolist() == [s2.get(r, 0) for r in names]
    # a start Python's int() reads but the native parse does not: the reference's own parse decides
    (d / "chr3~ 0012~40.psl").write_bytes(b"")
    s1, s2 = {}, {}
    assert define._roots(str(d), s1) == define._roots_py(str(d), s2) and s1 == s2
    assert define._root_names(str(d)) == define._roots_py(str(d))


class _Gather:
    """In-process all-gather over ranks run one after another: call c returns what every rank has
    contributed to call c so far (so the last rank sees everything)."""

    def __init__(self, rank, world, store):
        self.rank, self.world, self.store, self.calls = rank, world, store, 0

    def allgather_bytes(self, blob):
        import numpy as np

        c = self.store.setdefault(self.calls, {})
        self.calls += 1
        c[self.rank] = np.array(blob, dtype=np.uint8, copy=True)
        parts = [c.get(r, np.zeros(0, np.uint8)) for r in range(self.world)]
        return np.concatenate(parts), np.array([p.size for p in parts], dtype=np.int64)


def test_shared_roots_slices_equal_one_scan(tmp_path):
    """_shared_roots (rank 0 lists, every rank stats its slice) gives every rank the roots and sizes of
    one mando_list_roots scan; a slice not yet contributed (rank 0 runs first here) is stat'ed locally."""
    import numpy as np

    from mandalorion_amd import define

    d = tmp_path / "tmp_SS"
    d.mkdir()
    for i in range(1000):
        (d / f"chr{i % 7}~{i * 37}~{i * 37 + 5}.psl").write_bytes(b"y" * (i % 23))
    (d / "chr1~5~9.psl.bak").write_bytes(b"ab")
    sa = []
    ref = define._roots(str(d), size_array=sa)
    store = {}
    world = 3
    out = [define._shared_roots(str(d), _Gather(r, world, store)) for r in range(world)]
    for roots, sizes in out:
        assert roots == ref and np.array_equal(sizes, sa[0])
    assert [len(store[1][r]) for r in range(world)] == [8 * (len(ref) * (r + 1) // world - len(ref) * r // world)
                                                         for r in range(world)]
