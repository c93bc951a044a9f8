"""§8(f) row 2 on the GPU: SAM -> PSL by sam_kernel.hip (mando_sam_to_psl_device, emtrey.py:31-193) against
the reference's own outputs (tests/golden/sam_vectors.json, made by running emtrey here:
tests/golden/make_sam_vectors.py) and byte for byte against the host C++ restatement (sam.cpp) on a larger
synthetic SAM; Python repr() of the accuracy, the strand / revcomp rules and emtrey's failure cases."""
import hashlib
import os

import pytest

from mandalorion_amd import _lib, psl
from tests.test_sam import GOLD, _check, _gen

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("tag,mando", [("mando", True), ("plain", False)])
def test_gpu_sam_to_psl_matches_reference(tmp_path, tag, mando):
    m = _gen()
    sam = str(tmp_path / "in.sam")
    assert m.make_input(sam, with_cs=mando) == GOLD[tag + "_records"]
    out = str(tmp_path / "out.psl")
    n = psl.sam_to_psl(sam, out, mando=mando, device=0)
    assert n == GOLD[tag + "_psl"]["lines"]
    _check(out, GOLD[tag + "_psl"])


@pytest.mark.parametrize("mando", [True, False])
def test_gpu_equals_host_on_a_larger_sam(tmp_path, mando):
    m = _gen()
    sam = str(tmp_path / "big.sam")
    m.make_input(sam, n_reads=4000, seed=7, with_cs=mando)
    a, b = str(tmp_path / "gpu.psl"), str(tmp_path / "host.psl")
    na = psl.sam_to_psl(sam, a, mando=mando, device=0)
    nb = psl.sam_to_psl(sam, b, mando=mando, device=None, threads=4)
    assert na == nb > 1000
    assert hashlib.sha256(open(a, "rb").read()).hexdigest() == hashlib.sha256(open(b, "rb").read()).hexdigest()


def _one(tmp_path, cigar, tags, flag=0, seq=None, mando=True, device=0):
    seq = seq if seq is not None else "A" * 20
    sam = tmp_path / "x.sam"
    sam.write_text("@SQ\tSN:c\tLN:1000\n" + "\t".join(["r", str(flag), "c", "11", "60", cigar, "*", "0", "0", seq, "*"]
                                                      + tags) + "\n")
    out = str(tmp_path / "x.psl")
    psl.sam_to_psl(str(sam), out, mando=mando, device=device)
    return open(out).read().rstrip("\n").split("\t")


@pytest.mark.parametrize("m,nn", [(3, 0), (1, 99999), (1, 9999), (7, 42), (1, 6), (1000, 1), (2, 7), (333, 1000)])
def test_gpu_accuracy_is_python_repr(tmp_path, m, nn):
    f = _one(tmp_path, f"{m}M", [f"nn:i:{nn}", "NM:i:0", f"cs:Z:={'A' * m}"], seq="A" * m)
    assert f[21] == repr(m / (m + nn))


def test_gpu_strand_tag_and_revcomp(tmp_path):
    f = _one(tmp_path, "2S4M", ["cs:Z:=ACGT", "ts:A:-"], flag=16, seq="ACGTRn")
    assert f[8] == "+" and f[23] == "nYACGT" and f[11] == "2" and f[12] == "6"
    f = _one(tmp_path, "4M2H", ["cs:Z:=ACGT"], flag=0, seq="ACGT")
    assert f[8] == "+" and f[12] == "4" and f[10] == "6"
    # lists: I advances the query, D and N the target; = and X neither (emtrey's parseLine)
    f = _one(tmp_path, "3S5M2I4M3D6M100N2M1X", ["NM:i:5", "cs:Z:=ACGT"], seq="A" * 25)
    g = _one(tmp_path, "3S5M2I4M3D6M100N2M1X", ["NM:i:5", "cs:Z:=ACGT"], seq="A" * 25, device=None)
    assert f == g


def test_gpu_reference_failure_cases(tmp_path):
    with pytest.raises(_lib.MandoError):  # emtrey -m without a cs tag: NameError
        _one(tmp_path, "4M", ["NM:i:0"])
    with pytest.raises(_lib.MandoError):  # no aligned base: ZeroDivisionError
        _one(tmp_path, "4S", ["cs:Z:"])
    with pytest.raises(_lib.MandoError):  # a CIGAR number int() rejects
        _one(tmp_path, "4MxI", ["cs:Z:=ACGT"])
    sam = tmp_path / "y.sam"
    sam.write_text("@SQ\tSN:c\tLN:1000\nr\t0\tunknown\t1\t60\t4M\t*\t0\t0\tACGT\t*\tcs:Z:=ACGT\n")
    with pytest.raises(_lib.MandoError):  # chromosome without @SQ: KeyError
        psl.sam_to_psl(str(sam), str(tmp_path / "y.psl"), device=0)


def test_gpu_unmapped_and_header_only(tmp_path):
    sam = tmp_path / "z.sam"
    sam.write_text("@HD\tVN:1.6\n@SQ\tSN:c\tLN:1000\n\nr\t4\t*\t0\t0\t*\t*\t0\t0\tACGT\t*\n")
    out = str(tmp_path / "z.psl")
    assert psl.sam_to_psl(str(sam), out, device=0) == 0
    assert os.path.getsize(out) == 0
