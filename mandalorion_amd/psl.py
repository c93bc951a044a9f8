"""PSL ingest + locus split (libmando `mando_split_loci`): the part of module P that produces the D
module's input, i.e. `sort -k 14,14 -k 16,17n` of the clean PSL (/root/reference/Mando.py:343-349) and
get_chromosomes (/root/reference/utils/SpliceDefineConsensus.py:442-495), in one native pass."""
from __future__ import annotations

import ctypes
import os

from . import _lib


def split_loci(clean_psl: str, tmp_ss: str, sort_lines: bool = True, sorted_out: str | None = None) -> tuple[int, int]:
    """Writes <tmp_ss>/<chrom>~<start>~<end>.psl per locus; returns (records, loci)."""
    os.makedirs(tmp_ss, exist_ok=True)
    nr = ctypes.c_int64()
    nl = ctypes.c_int64()
    _lib.check(_lib.load().mando_split_loci(clean_psl.encode(), tmp_ss.encode(), 1 if sort_lines else 0,
                                            sorted_out.encode() if sorted_out else None, ctypes.byref(nr),
                                            ctypes.byref(nl)))
    return nr.value, nl.value
