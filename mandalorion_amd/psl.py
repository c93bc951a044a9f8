"""Module P natively (libmando): SAM -> PSL (`mando_sam_to_psl`, emtrey.py -m), clean_psl
(`mando_clean_psl`, /root/reference/utils/SpliceDefineConsensus.py:14-92) and the locus split that produces
the D module's input (`mando_split_loci`: `sort -k 14,14 -k 16,17n` of the clean PSL,
/root/reference/Mando.py:343-349, and get_chromosomes, SpliceDefineConsensus.py:442-495)."""
from __future__ import annotations

import ctypes
import os

from . import _lib


def split_loci(clean_psl: str, tmp_ss: str, sort_lines: bool = True, sorted_out: str | None = None,
               device: int | None | str = "auto") -> tuple[int, int]:
    """Writes <tmp_ss>/<chrom>~<start>~<end>.psl per locus; returns (records, loci).  device: a GPU
    ordinal parses and sorts there (mando_split_loci_device, psl_kernel.hip); "auto" uses GPU 0 when one
    is visible; None the host C++ (mando_split_loci).  Both write the same bytes."""
    os.makedirs(tmp_ss, exist_ok=True)
    nr = ctypes.c_int64()
    nl = ctypes.c_int64()
    lib = _lib.load()
    if device == "auto":
        device = 0 if _lib.device_count() > 0 else None
    srt = sorted_out.encode() if sorted_out else None
    if device is not None:
        ctx = _lib.context(int(device), slot=4)
        _lib.check(lib.mando_split_loci_device(ctx.handle, clean_psl.encode(), tmp_ss.encode(), 1 if sort_lines else 0,
                                               srt, ctypes.byref(nr), ctypes.byref(nl)))
    else:
        _lib.check(lib.mando_split_loci(clean_psl.encode(), tmp_ss.encode(), 1 if sort_lines else 0, srt,
                                        ctypes.byref(nr), ctypes.byref(nl)))
    return nr.value, nl.value


def sam_to_psl(sam: str, psl: str, mando: bool = True, threads: int = 0, device: int | None | str = "auto") -> int:
    """emtrey.py -i sam -o psl [-m] (/root/reference/emtrey.py:31-193); returns PSL lines written.
    Raises MandoError where emtrey raises (unknown chromosome, missing cs tag in -m mode, zero-length
    alignment, malformed CIGAR).  device: a GPU ordinal runs the conversion there
    (mando_sam_to_psl_device, sam_kernel.hip); "auto" uses GPU 0 when one is visible; None the host C++
    threads (mando_sam_to_psl).  Both write the same bytes."""
    n = ctypes.c_int64()
    lib = _lib.load()
    if device == "auto":
        device = 0 if _lib.device_count() > 0 else None
    if device is not None:
        ctx = _lib.context(int(device), slot=4)
        _lib.check(lib.mando_sam_to_psl_device(ctx.handle, sam.encode(), psl.encode(), 1 if mando else 0,
                                               ctypes.byref(n)))
    else:
        _lib.check(lib.mando_sam_to_psl(sam.encode(), psl.encode(), 1 if mando else 0, int(threads),
                                        ctypes.byref(n)))
    return n.value


def clean_psl(psl_file: str, clean_psl_file: str, primary: bool) -> int:
    """SpliceDefineConsensus.clean_psl (same argument order); returns lines written."""
    n = ctypes.c_int64()
    _lib.check(_lib.load().mando_clean_psl(psl_file.encode(), clean_psl_file.encode(), 1 if primary else 0,
                                           ctypes.byref(n)))
    return n.value
