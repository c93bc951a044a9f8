"""§8(f) row 3 on the GPU: module F (filterIsoforms.py) with look_for_contained_isoforms' candidate search on
the device (modf_kernel.hip, mando_filter_isoforms_device) against the reference's own outputs for the
fixture inputs (tests/golden/fq_vectors.json) and byte for byte against the host path
(mando_filter_isoforms) on larger synthetic inputs (tests/modf_synth.py: shared exon sets per locus, both
strands, A-rich ends, a polyA whitelist) over internal ratios and splice windows that make every reason
fire."""
import os
import shutil

import pytest

from mandalorion_amd import modules
from tests import modf_synth
from tests.test_module_fq import GOLD, _digest, _gen, _params

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("multi", [0, 1])
def test_gpu_module_f_matches_reference(tmp_path, multi):
    m = _gen()
    d = str(tmp_path)
    assert m.make_input(d) == GOLD["isoforms"]
    shutil.copy(os.path.join(d, "iso.sam"), os.path.join(d, "Isoforms.aligned.out.sam"))
    gold = GOLD[f"multi{multi}"]
    n = modules.module_f(d, os.path.join(d, "Isoform_Consensi.fasta"), os.path.join(d, "genome.fa"),
                         _params(multi, gold["internal_ratio"]), threads=4, device=0)
    assert n == gold["Isoforms.filtered.clean.psl"]["lines"]
    for f in ("Isoforms.aligned.out.clean.psl", "Isoforms.filtered.fasta", "Isoforms.filtered.clean.psl",
              "Isoforms.filtered.clean.gtf"):
        assert _digest(os.path.join(d, f)) == gold[f], f
    got = m.normalise(open(os.path.join(d, "filter_reasons.txt")).read().split("\n")[:-1])
    assert got == gold["reasons"]


@pytest.mark.parametrize("seed,internal_ratio,sw,multi", [(1, 1.0, 1, 0), (2, 0.3, 1, 0), (3, 0.3, 5, 1),
                                                            (4, 1.0, 5, 0), (5, 0.3, 0, 0)])
def test_gpu_module_f_equals_host(tmp_path, seed, internal_ratio, sw, multi):
    d = str(tmp_path)
    assert modf_synth.write_inputs(d, n_loci=600, seed=seed) > 1000
    p = modules.FilterParams.default()
    p.threads = 4
    p.internal_ratio = internal_ratio
    p.splice_window = sw
    p.multi_exon_only = multi
    outs = {}
    for dev in (0, None):
        o = os.path.join(d, f"out_{dev}")
        n = modules.filter_isoforms(p, os.path.join(d, "Isoform_Consensi.fasta"), os.path.join(d, "genome.fa"),
                                    os.path.join(d, "clean.psl"), os.path.join(d, "polyAWhiteList.bed"),
                                    o + ".fa", o + ".psl", o + ".reasons", device=dev)
        outs[dev] = (n, open(o + ".fa", "rb").read(), open(o + ".psl", "rb").read(), open(o + ".reasons", "rb").read())
    assert outs[0] == outs[None]
    reasons = outs[0][3].decode()
    assert "internal to" in reasons and " filtered because at " in reasons
    if internal_ratio < 1.0 and sw > 0:
        assert "almost identical" in reasons
