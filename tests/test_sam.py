"""§8(f) row 2: SAM -> PSL (mando_sam_to_psl, emtrey.py -m) and clean_psl (mando_clean_psl) against the
reference's own outputs on the same synthetic SAM (tests/golden/make_sam_vectors.py; fixture
tests/golden/sam_vectors.json: per-line and whole-file sha256), plus the float formatting and the
reference's failure cases."""
import hashlib
import importlib.util
import json
import os

import pytest

from mandalorion_amd import _lib, psl

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = json.load(open(os.path.join(HERE, "golden", "sam_vectors.json")))


def _gen():
    spec = importlib.util.spec_from_file_location("msam", os.path.join(HERE, "golden", "make_sam_vectors.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _check(path, gold):
    data = open(path, "rb").read()
    lines = data.split(b"\n")[:-1]
    got = [hashlib.sha256(l).hexdigest()[:16] for l in lines]
    assert len(lines) == gold["lines"]
    bad = [i for i, (a, b) in enumerate(zip(got, gold["line_sha"])) if a != b]
    assert not bad, f"lines differing from the reference: {bad[:10]}"
    assert hashlib.sha256(data).hexdigest() == gold["sha256"]


@pytest.mark.parametrize("tag,mando", [("mando", True), ("plain", False)])
@pytest.mark.parametrize("threads", [1, 3])
def test_sam_to_psl_matches_reference(tmp_path, tag, mando, threads):
    m = _gen()
    sam = str(tmp_path / "in.sam")
    assert m.make_input(sam, with_cs=mando) == GOLD[tag + "_records"]
    out = str(tmp_path / "out.psl")
    n = psl.sam_to_psl(sam, out, mando=mando, threads=threads)
    assert n == GOLD[tag + "_psl"]["lines"]
    _check(out, GOLD[tag + "_psl"])
    for primary in (1, 0):
        clean = str(tmp_path / f"clean{primary}.psl")
        assert psl.clean_psl(out, clean, bool(primary)) == GOLD[f"{tag}_clean_primary{primary}"]["lines"]
        _check(clean, GOLD[f"{tag}_clean_primary{primary}"])


def _one(tmp_path, cigar, tags, flag=0, seq=None, mando=True):
    seq = seq if seq is not None else "A" * 20
    sam = tmp_path / "x.sam"
    sam.write_text("@SQ\tSN:c\tLN:1000\n" + "\t".join(["r", str(flag), "c", "11", "60", cigar, "*", "0", "0", seq, "*"]
                                                      + tags) + "\n")
    out = str(tmp_path / "x.psl")
    psl.sam_to_psl(str(sam), out, mando=mando)
    return open(out).read().rstrip("\n").split("\t")


@pytest.mark.parametrize("m,nn", [(3, 0), (1, 99999), (1, 9999), (7, 42), (1, 6), (1000, 1)])
def test_accuracy_is_python_repr(tmp_path, m, nn):
    f = _one(tmp_path, f"{m}M", [f"nn:i:{nn}", "NM:i:0", f"cs:Z:={'A' * m}"], seq="A" * m)
    assert f[21] == repr(m / (m + nn))


def test_strand_tag_and_revcomp(tmp_path):
    # flag 16 -> '-' and the read reverse-complemented (IUPAC, case kept); ts:A:- flips the strand back
    f = _one(tmp_path, "2S4M", ["cs:Z:=ACGT", "ts:A:-"], flag=16, seq="ACGTRn")
    assert f[8] == "+" and f[23] == "nYACGT" and f[11] == "2" and f[12] == "6"
    f = _one(tmp_path, "4M2H", ["cs:Z:=ACGT"], flag=0, seq="ACGT")
    assert f[8] == "+" and f[12] == "4" and f[10] == "6"


def test_reference_failure_cases(tmp_path):
    with pytest.raises(_lib.MandoError):  # emtrey -m without a cs tag: NameError
        _one(tmp_path, "4M", ["NM:i:0"])
    with pytest.raises(_lib.MandoError):  # no aligned base: ZeroDivisionError
        _one(tmp_path, "4S", ["cs:Z:"])
    sam = tmp_path / "y.sam"
    sam.write_text("@SQ\tSN:c\tLN:1000\nr\t0\tunknown\t1\t60\t4M\t*\t0\t0\tACGT\t*\tcs:Z:=ACGT\n")
    with pytest.raises(_lib.MandoError):  # chromosome without @SQ: KeyError
        psl.sam_to_psl(str(sam), str(tmp_path / "y.psl"))


def test_clean_psl_merges_small_gaps(tmp_path):
    line = "\t".join(["90", "0", "0", "0", "0", "0", "0", "0", "+", "r", "100", "5", "95", "c", "1000", "100",
                      "420", "4", "30,20,20,20,", "5,35,55,75,", "100,135,160,400,"])
    src = tmp_path / "a.psl"
    src.write_text(line + "\n" + line.replace("\tr\t", "\tr2\t") + "\n" + line + "\n")
    dst = str(tmp_path / "b.psl")
    assert psl.clean_psl(str(src), dst, True) == 2
    f = open(dst).read().split("\n")[0].split("\t")
    # gaps 5 and 5 (< 10) merge blocks 1-3 into 80 nt; the 220-nt gap stays
    assert f[17:21] == ["2", "80,20,", "5,85,", "100,400,"]


def test_mando_cli_module_P_from_sam(tmp_path):
    """`Mando.py -M P` with tmp/mm2Alignments.sam: emtrey -m + clean_psl(primary) outputs equal the
    reference's, then the sorted PSL is split into loci covering every clean record."""
    from mandalorion_amd import mando

    tmp = tmp_path / "tmp"
    tmp.mkdir()
    _gen().make_input(str(tmp / "mm2Alignments.sam"), with_cs=True)
    assert mando.main(["-p", str(tmp_path), "-M", "P", "-t", "4"]) == 0
    _check(str(tmp / "mm2Alignments.psl"), GOLD["mando_psl"])
    _check(str(tmp / "mm2Alignments.clean.psl"), GOLD["mando_clean_primary1"])
    n = sum(len(open(tmp / "tmp_SS" / f).read().splitlines()) for f in os.listdir(tmp / "tmp_SS"))
    assert n == GOLD["mando_clean_primary1"]["lines"]
