"""`python -m mandalorion_amd.abpoa` — the abpoa-argv parity vehicle.

The reference calls `abpoa -M 5 -r 0 [-S] root.fasta` (SpliceDefineConsensus.py:915-919) and keeps the
last FASTA record of stdout.  CPU: argv and FASTA handling.  GPU: the tool's consensus equals the CPU
restatement's (oracle/poa_ref.c) for plain and `-S` groups.
"""
from __future__ import annotations

import io
import contextlib

import pytest

from mandalorion_amd import abpoa, synth


def test_argv_maps_onto_poa_params():
    a = abpoa.parser().parse_args(["-M", "5", "-r", "0", "-S", "x.fa"])
    p = abpoa.params_from(a)
    assert (p.match, p.mismatch, p.gap_open1, p.gap_ext1, p.gap_open2, p.gap_ext2) == (5, 4, 4, 2, 24, 1)
    assert (p.band_b, round(p.band_f, 4), p.seeding, p.k, p.w, p.min_w) == (10, 0.01, 1, 19, 10, 500)
    a = abpoa.parser().parse_args(["-M", "5", "-r", "0", "x.fa"])
    assert abpoa.params_from(a).seeding == 0


def test_fasta_reader(tmp_path):
    f = tmp_path / "in.fa"
    f.write_text(">r1 desc\nACGT\nAC\n>r2\n\n>r3\nGG\n")
    assert abpoa.read_fasta(str(f)) == [("r1", "ACGTAC"), ("r2", ""), ("r3", "GG")]


def test_only_consensus_output(tmp_path):
    f = tmp_path / "in.fa"
    f.write_text(">r1\nACGT\n")
    assert abpoa.main(["-r", "1", str(f)]) == 2


def _cli(args):
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        assert abpoa.main(args) == 0
    lines = buf.getvalue().splitlines()
    assert lines[0] == ">Consensus_sequence" and len(lines) == 2
    return lines[1]


@pytest.mark.gpu
@pytest.mark.parametrize("seeded", [False, True])
def test_cli_equals_oracle(gpu_ctx, tmp_path, seeded):
    from oracle import poa as opoa

    length = (8200, 8600) if seeded else (2500, 3000)
    reads = synth.read_groups(1, length, 12, seed=31 + seeded)[1][0]
    f = tmp_path / "root.fasta"
    f.write_text("".join(f">read{i}\n{s}\n" for i, s in enumerate(reads)))
    args = ["-M", "5", "-r", "0"] + (["-S"] if seeded else []) + [str(f)]
    assert _cli(args) == opoa.consensus_batch([reads], seeding=[seeded])[0]
