"""§8(f) row 1 on the GPU: PSL ingest + locus split with the parse and the sort on the device
(psl_kernel.hip, mando_split_loci_device) against the reference's own split of the same input
(tests/golden/split_vectors.json: GNU sort + get_chromosomes run here) and byte for byte against the host
restatement (psl.cpp) on a larger shuffled PSL with duplicated lines and (chromosome, start) ties."""
import hashlib
import os
import random

import pytest

from mandalorion_amd import psl, synth
from tests.test_split import GOLD, _make_input

pytestmark = pytest.mark.gpu


def _digest_dir(d):
    return {f: hashlib.sha256(open(os.path.join(d, f), "rb").read()).hexdigest() for f in sorted(os.listdir(d))}


def test_gpu_split_matches_reference(tmp_path):
    src = str(tmp_path / "clean.psl")
    assert _make_input(src) == GOLD["records"]
    srt = str(tmp_path / "clean.sorted.psl")
    nrec, nloc = psl.split_loci(src, str(tmp_path / "tmp_SS"), sort_lines=True, sorted_out=srt, device=0)
    assert nrec == GOLD["records"] and nloc == len(GOLD["loci"])
    assert hashlib.sha256(open(srt, "rb").read()).hexdigest() == GOLD["sorted_sha256"]
    assert _digest_dir(tmp_path / "tmp_SS") == GOLD["loci"]


def test_gpu_split_presorted_input(tmp_path):
    src = str(tmp_path / "clean.psl")
    _make_input(src)
    srt = str(tmp_path / "s1.psl")
    psl.split_loci(src, str(tmp_path / "a"), sort_lines=True, sorted_out=srt, device=0)
    psl.split_loci(srt, str(tmp_path / "b"), sort_lines=False, device=0)
    assert _digest_dir(tmp_path / "a") == _digest_dir(tmp_path / "b")


def test_gpu_split_equals_host_on_a_larger_shuffled_psl(tmp_path):
    ss = tmp_path / "ss"
    synth.write_loci(str(ss), 300, reads=(20, 40), seed=11, rev_frac=0.5)
    lines = []
    for f in sorted(os.listdir(ss)):
        lines += open(ss / f, "rb").read().splitlines()
    rng = random.Random(3)
    # exact duplicates and (chromosome, start) ties with different bytes (GNU sort's whole-line key)
    extra = []
    for ln in rng.sample(lines, 200):
        extra.append(ln)
        f = ln.split(b"\t")
        f[0] = str(int(f[0]) + rng.randrange(1, 50)).encode()
        extra.append(b"\t".join(f))
    lines += extra
    rng.shuffle(lines)
    src = tmp_path / "in.psl"
    src.write_bytes(b"\n".join(lines) + b"\n")
    a, b = tmp_path / "gpu", tmp_path / "host"
    na = psl.split_loci(str(src), str(a), sort_lines=True, sorted_out=str(tmp_path / "a.psl"), device=0)
    nb = psl.split_loci(str(src), str(b), sort_lines=True, sorted_out=str(tmp_path / "b.psl"), device=None)
    assert na == nb and na[0] == len(lines)
    assert open(tmp_path / "a.psl", "rb").read() == open(tmp_path / "b.psl", "rb").read()
    assert _digest_dir(a) == _digest_dir(b)


def test_gpu_split_rejects_what_the_host_rejects(tmp_path):
    from mandalorion_amd import _lib

    src = tmp_path / "bad.psl"
    src.write_text("1\t2\t3\n")  # fewer than 17 fields
    with pytest.raises(_lib.MandoError):
        psl.split_loci(str(src), str(tmp_path / "o"), device=0)
    with pytest.raises(_lib.MandoError):
        psl.split_loci(str(src), str(tmp_path / "o2"), device=None)
