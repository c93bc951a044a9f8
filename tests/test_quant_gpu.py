"""§8(f) row 4 on the GPU: module Q (assignReadsToIsoforms.py:27-105) with its joins on the device
(quant_kernel.hip, mando_quantify_device) against the reference's own tables for the fixture inputs
(tests/golden/fq_vectors.json) and byte for byte against the host path (mando_quantify) on larger inputs:
several read files (FASTA, FASTQ, gzip), read names repeated across files (the dict keeps the last
file's), reads2isoforms lines with surrounding blanks, duplicated and absent isoforms."""
import gzip
import hashlib
import os
import random
import shutil

import pytest

from mandalorion_amd import _lib, modules
from tests.test_module_fq import GOLD, _gen, _params

pytestmark = pytest.mark.gpu

OUTS = ("Isoforms.filtered.clean.quant", "Isoforms.filtered.clean.tpm")


def test_gpu_quant_matches_reference(tmp_path):
    m = _gen()
    d = str(tmp_path)
    m.make_input(d)
    shutil.copy(os.path.join(d, "iso.sam"), os.path.join(d, "Isoforms.aligned.out.sam"))
    modules.module_f(d, os.path.join(d, "Isoform_Consensi.fasta"), os.path.join(d, "genome.fa"), _params(0, 1.0))
    files = [os.path.join(d, "a.fasta"), os.path.join(d, "b.fasta")]
    modules.quantify(d, files, device=0)
    for f in OUTS:
        data = open(os.path.join(d, f)).read()
        assert data.split("\n")[0] == "Isoform\t" + "".join(x + "\t" for x in files)
        body = "\n".join(data.split("\n")[1:])
        assert hashlib.sha256(body.encode()).hexdigest() == GOLD["multi0"][f]["sha256_body"], f
        assert data.count("\n") == GOLD["multi0"][f]["lines"]


def _write_inputs(d, n_reads=60000, n_iso=3000, seed=5):
    rng = random.Random(seed)
    names = [f"read_{i:07d}_{rng.randrange(1 << 30):x}" for i in range(n_reads)]
    # three read files: FASTA (multi-line sequences), FASTQ (4-line records), gzip FASTA; 5 % of the
    # names appear again in a later file (the dict keeps the later file)
    parts = [names[: n_reads // 3], names[n_reads // 3: 2 * n_reads // 3], names[2 * n_reads // 3:]]
    dup = rng.sample(names[: 2 * n_reads // 3], n_reads // 20)
    parts[2] = parts[2] + dup
    seq = lambda: "".join(rng.choice("ACGT") for _ in range(rng.randrange(20, 90)))  # noqa: E731
    with open(os.path.join(d, "r1.fa"), "w") as fh:
        for nm in parts[0]:
            s = seq()
            fh.write(f">{nm} some description\n{s[:40]}\n{s[40:]}\n" if len(s) > 40 else f">{nm}\n{s}\n")
    with open(os.path.join(d, "r2.fq"), "w") as fh:
        for nm in parts[1]:
            s = seq()
            fh.write(f"@{nm}\tx\n{s}\n+\n{'I' * len(s)}\n")
    with gzip.open(os.path.join(d, "r3.fa.gz"), "wt") as fh:
        for nm in parts[2]:
            fh.write(f">{nm}\n{seq()}\n")
    isos = [f"Isoform{i}_{rng.randrange(1, 400)}" for i in range(n_iso)]
    with open(os.path.join(d, "reads2isoforms.txt"), "w") as fh:
        for nm in names:
            lead = " " if rng.random() < 0.01 else ""
            fh.write(f"{lead}{nm}\t{rng.choice(isos)}\n")
    used = sorted({ln.split("\t")[1].strip() for ln in open(os.path.join(d, "reads2isoforms.txt"))})
    psl = rng.sample(used, len(used) // 2)
    psl += rng.sample(psl, 20)  # an isoform listed twice gets two rows
    with open(os.path.join(d, "Isoforms.filtered.clean.psl"), "w") as fh:
        for nm in psl:
            f = ["0"] * 21
            f[9] = nm
            fh.write("\t".join(f) + "\n")
    return [os.path.join(d, x) for x in ("r1.fa", "r2.fq", "r3.fa.gz")]


def test_gpu_quant_equals_host(tmp_path):
    a, b = tmp_path / "gpu", tmp_path / "host"
    a.mkdir()
    files = _write_inputs(str(a))
    shutil.copytree(a, b, dirs_exist_ok=True)
    files_b = [f.replace(str(a), str(b)) for f in files]
    modules.quantify(str(a), files, device=0)
    modules.quantify(str(b), files_b, device=None)
    for f in OUTS:
        ga, hb = open(a / f).read(), open(b / f).read()
        # the header names the files (different folders); the rows must be identical
        assert ga.split("\n")[1:] == hb.split("\n")[1:], f
        assert ga.count("\n") > 1000


@pytest.mark.parametrize("case", ["missing_read", "missing_isoform", "one_field"])
def test_gpu_quant_errors_like_host(tmp_path, case):
    d = tmp_path
    (d / "a.fa").write_text(">r1\nACGT\n>r2\nAC\n")
    r2i = {"missing_read": "r1\tIso_1\nr9\tIso_1\n", "missing_isoform": "r1\tIso_1\n", "one_field": "r1\tIso_1\nr2\n"}[case]
    (d / "reads2isoforms.txt").write_text(r2i)
    iso = "Iso_2" if case == "missing_isoform" else "Iso_1"
    (d / "Isoforms.filtered.clean.psl").write_text("\t".join(["0"] * 9 + [iso] + ["0"] * 11) + "\n")
    for dev in (0, None):
        with pytest.raises(_lib.MandoError):
            modules.quantify(str(d), [str(d / "a.fa")], device=dev)
