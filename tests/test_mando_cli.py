"""`Mando.py -M D` (the CLI entry, /root/reference/Mando.py:362-402) on BASELINE configs[0]: 100 synthetic
loci x 5 reads x ~1 kb, against the unmodified reference run on the same loci
(tests/golden/define_vectors.json "config1", made by tests/golden/make_define_vectors.py with
Mando.py:382-399's defineIsoforms argv: -c 0.1 -g None -w 1 -m 2 -W 0 -n 8 -j <default> -u 10 -d 50).

The module writes <p>/tmp/Isoform_Consensi.fasta and <p>/tmp/reads2isoforms.txt, and Mando.py:400 copies
the latter to <p>/Mando_isoforms.read_stat.txt.  All three must equal the reference's bytes.

* CPU (not gpu): the CLI in-process with the oracle's clustering, orientation and POA injected into the
  driver (the CLI plumbing: argument mapping, input checks, the read_stat copy).
* GPU: the repo-root `Mando.py -M D` as a subprocess, i.e. the product path (HIP kernels) end to end.
"""
from __future__ import annotations

import functools
import hashlib
import json
import os
import subprocess
import sys

import pytest

from mandalorion_amd import synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = json.load(open(os.path.join(ROOT, "tests", "golden", "define_vectors.json")))
C1 = GOLD["datasets"]["config1"]


def sha(path):
    return hashlib.sha256(open(path, "rb").read()).hexdigest()


def _layout(tmp_path) -> str:
    """<p>/tmp/tmp_SS/*.psl (module P's output) and the non-empty clean sorted PSL Mando.py:370-375 checks."""
    p = str(tmp_path / "mando_out")
    tmp = os.path.join(p, "tmp")
    spec = dict(C1["synth"])
    n = spec.pop("n_loci")
    recs = synth.write_loci(os.path.join(tmp, "tmp_SS"), n, threads=4, **spec)
    assert recs == C1["inputs"]["records"]
    files = sorted(os.listdir(os.path.join(tmp, "tmp_SS")))
    assert {f: sha(os.path.join(tmp, "tmp_SS", f)) for f in files} == C1["inputs"]["psl_sha256"]
    with open(os.path.join(tmp, "mm2Alignments.clean.sorted.psl"), "wb") as out:
        for f in files:
            out.write(open(os.path.join(tmp, "tmp_SS", f), "rb").read())
    return p


def _check(p):
    ref = C1["reference"]
    tmp = os.path.join(p, "tmp")
    assert sha(os.path.join(tmp, "reads2isoforms.txt")) == ref["reads2isoforms_sha256"]
    assert sha(os.path.join(tmp, "Isoform_Consensi.fasta")) == ref["isoform_consensi_sha256"]
    assert sha(os.path.join(p, "Mando_isoforms.read_stat.txt")) == ref["reads2isoforms_sha256"]
    assert os.path.exists(os.path.join(tmp, "polyAWhiteList.bed"))
    headers = [l[1:].rstrip("\n") for l in open(os.path.join(tmp, "Isoform_Consensi.fasta")) if l.startswith(">")]
    assert headers == ref["isoform_headers"]
    # the metrics line next to Mando.log: one JSON object per run
    m = json.loads(open(os.path.join(p, "Mando.metrics.jsonl")).read().splitlines()[-1])
    assert (m["module"], m["ranks"], m["records_rank0"]) == ("D", 1, C1["inputs"]["records"])
    assert m["isoforms_rank0"] == len(ref["isoform_headers"]) and m["wall_s"] > 0
    return m


def test_mando_cli_module_d_config1_with_oracle(tmp_path, monkeypatch):
    from mandalorion_amd import define, mando
    from oracle import cluster as ocl
    from oracle import orient as oref
    from oracle import poa as opoa

    p = _layout(tmp_path)
    calls = []
    real = define.define_isoforms

    def injected(*a, **kw):
        calls.append(kw)
        return real(*a, orient_fn=lambda s, o, g: oref.orient_packed(s, o, g),
                    consensus_fn=lambda s, o, g, sd: opoa.consensus_packed(s, o, g, seeding=sd),
                    cluster_fn=ocl.cluster_loci, **kw)

    monkeypatch.setattr(define, "define_isoforms", injected)
    assert mando.main(["-M", "D", "-p", p, "--seed", str(GOLD["seed"])]) == 0
    # Mando.py:382-399's argv, as keyword arguments of the driver
    kw = calls[0]
    assert (kw["cutoff"], kw["genome_file"], kw["splice_site_width"], kw["minimum_read_count"]) == (0.1, "None", 1, 2)
    assert (kw["white_list_polyA"], kw["threads"], kw["upstream_buffer"], kw["downstream_buffer"]) == (["0"], 8, 10, 50)
    assert kw["junctions"] == "gtag,gcag,atac,ctac,ctgc,gtat"
    _check(p)


def test_mando_cli_module_d_missing_input_is_skipped(tmp_path, capsys):
    """Mando.py:370-380: no clean sorted PSL -> the module reports and writes nothing."""
    from mandalorion_amd import mando

    p = str(tmp_path / "empty")
    assert mando.main(["-M", "D", "-p", p]) == 0
    assert "clean sorted psl file missing or empty" in capsys.readouterr().out
    assert not os.path.exists(os.path.join(p, "tmp", "Isoform_Consensi.fasta"))


@pytest.mark.gpu
def test_mando_cli_module_d_config1_gpu(tmp_path):
    p = _layout(tmp_path)
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "Mando.py"), "-M", "D", "-p", p, "--seed", str(GOLD["seed"])],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    m = _check(p)
    assert m["poa_kernel_ms"] > 0 and m["dp_cells"] > 0 and 0 < m["poa_hbm_roofline_frac"] < 1
