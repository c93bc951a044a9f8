"""`abpoa`-argv-compatible consensus tool over libmando (SURVEY.md §8(b) "Optional parity vehicle").

The reference shells out once per isoform (/root/reference/utils/SpliceDefineConsensus.py:915-919):

    abpoa -M 5 -r 0 [-S] root.fasta > root.consensus.fasta 2> abpoa.messages

and keeps the last FASTA record of stdout (SDC:922-923).  This module accepts the same argv, reads the
FASTA (every record, in file order: the POA input order), runs one group through `mando_poa_batch` on
the GPU and prints `>Consensus_sequence\\n<consensus>\\n`, so the unmodified reference
`defineIsoforms.py -a <this tool>` can drive the MI355X POA.  Scoring options abPOA v1.4.1 exposes
(-M -X -O -E -b -f -k -w -m) map onto mando_poa_params; `-r` must be 0 (consensus FASTA), the only
output the reference asks for.  There is no CPU path: without a gfx950 device the tool fails loudly.

    python -m mandalorion_amd.abpoa -M 5 -r 0 [-S] reads.fa
"""
from __future__ import annotations

import argparse
import sys

from . import _lib, poa


def read_fasta(path: str) -> list[tuple[str, str]]:
    """All records (name = header up to the first whitespace; multi-line sequences joined)."""
    recs: list[tuple[str, str]] = []
    name, seq = None, []
    with open(path) as fh:
        for line in fh:
            line = line.rstrip("\r\n")
            if line.startswith(">"):
                if name is not None:
                    recs.append((name, "".join(seq)))
                name, seq = line[1:].split()[0] if line[1:].split() else "", []
            elif name is not None:
                seq.append(line.strip())
    if name is not None:
        recs.append((name, "".join(seq)))
    return recs


def parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(prog="abpoa", description="abPOA-compatible consensus on MI355X (libmando)")
    ap.add_argument("-M", "--match", type=int, default=2)
    ap.add_argument("-X", "--mismatch", type=int, default=4)
    ap.add_argument("-O", "--gap-open", type=str, default="4,24")
    ap.add_argument("-E", "--gap-ext", type=str, default="2,1")
    ap.add_argument("-b", "--extra-b", type=int, default=10)
    ap.add_argument("-f", "--extra-f", type=float, default=0.01)
    ap.add_argument("-S", "--seeding", action="store_true")
    ap.add_argument("-k", "--k-mer", type=int, default=19)
    ap.add_argument("-w", "--window", type=int, default=10)
    ap.add_argument("-m", "--min-poa-win", type=int, default=500)
    ap.add_argument("-r", "--result", type=int, default=0)
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("input")
    return ap


def params_from(a) -> _lib.PoaParams:
    p = _lib.PoaParams.defaults()
    o = [int(x) for x in a.gap_open.split(",")]
    e = [int(x) for x in a.gap_ext.split(",")]
    p.match, p.mismatch = a.match, a.mismatch
    p.gap_open1, p.gap_ext1 = o[0], e[0]
    if len(o) > 1 and len(e) > 1:
        p.gap_open2, p.gap_ext2 = o[1], e[1]
    p.band_b, p.band_f = a.extra_b, a.extra_f
    p.seeding, p.k, p.w, p.min_w = int(a.seeding), a.k_mer, a.window, a.min_poa_win
    return p


def main(argv: list[str] | None = None) -> int:
    a = parser().parse_args(sys.argv[1:] if argv is None else argv)
    if a.result != 0:
        print("abpoa (mandalorion_amd): only -r 0 (consensus FASTA) is supported", file=sys.stderr)
        return 2
    recs = read_fasta(a.input)
    if not recs:
        return 0
    cons = poa.poa_consensus_batch([[s for _, s in recs]], params=params_from(a), seeding=[a.seeding],
                                   device=a.device)[0]
    sys.stdout.write(f">Consensus_sequence\n{cons}\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
