"""Modules F and Q natively (libmando, csrc/module_f.cpp): the consumers of the D module's consensi
(SURVEY.md §8(f) rows 3-4).

- Module F: filterIsoforms.py (/root/reference/filterIsoforms.py:456-510). The consensi are aligned by
  an external aligner (minimap2, as in the reference), then filter_sam -> SAM->PSL (emtrey, plain
  mode) -> clean_psl(primary=False) -> per-chromosome filters -> Isoforms.filtered.fasta,
  Isoforms.filtered.clean.psl, Isoforms.filtered.clean.gtf, filter_reasons.txt.
- Module Q: assignReadsToIsoforms.py:27-105 -> Isoforms.filtered.clean.quant / .tpm.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

from . import _lib, psl


class FilterParams(ctypes.Structure):
    """include/mando.h mando_filter_params (filterIsoforms.py arguments)."""
    _fields_ = [("minimum_ratio", ctypes.c_double), ("minimum_reads", ctypes.c_double),
                ("internal_ratio", ctypes.c_double), ("Acutoff", ctypes.c_double),
                ("overhangs", ctypes.c_int32 * 4), ("splice_window", ctypes.c_int32),
                ("downstream_buffer", ctypes.c_int32), ("minimum_isoform_length", ctypes.c_int32),
                ("multi_exon_only", ctypes.c_int32), ("threads", ctypes.c_int32)]

    @classmethod
    def default(cls) -> "FilterParams":
        p = cls()
        _lib.load().mando_filter_default_params(ctypes.byref(p))
        return p


def filter_sam(sam: str, out: str) -> int:
    n = ctypes.c_int64()
    _lib.check(_lib.load().mando_filter_sam(sam.encode(), out.encode(), ctypes.byref(n)))
    return n.value


def psl_to_gtf(psl_file: str, gtf_file: str) -> None:
    _lib.check(_lib.load().mando_psl_to_gtf(psl_file.encode(), gtf_file.encode()))


def _device(device):
    return (0 if _lib.device_count() > 0 else None) if device == "auto" else device


def filter_isoforms(params: FilterParams, isoform_fasta: str, genome_fasta: str, clean_psl: str,
                    whitelist_bed: str | None, out_fasta: str, out_psl: str, reasons: str | None = None,
                    device="auto") -> int:
    """filterIsoforms.process_chr over every chromosome + write_isoforms.  device: a GPU ordinal runs the
    containment search there (mando_filter_isoforms_device), None the host C++ (mando_filter_isoforms),
    "auto" GPU 0 when one is visible; both write the same bytes."""
    n = ctypes.c_int64()
    enc = lambda x: x.encode() if x else None  # noqa: E731
    args = (ctypes.byref(params), enc(isoform_fasta), enc(genome_fasta), enc(clean_psl), enc(whitelist_bed),
            enc(out_fasta), enc(out_psl), enc(reasons), ctypes.byref(n))
    dev = _device(device)
    lib = _lib.load()
    if dev is None:
        _lib.check(lib.mando_filter_isoforms(*args))
    else:
        _lib.check(lib.mando_filter_isoforms_device(_lib.context(int(dev), slot=4).handle, *args))
    return n.value


def module_f(path: str, isoform_fasta: str, genome_fasta: str, params: FilterParams,
             minimap2: str | None = None, threads: int = 8, device="auto") -> int:
    """filterIsoforms.main (filterIsoforms.py:456-510) in `path`.  The alignment of the consensi is the
    reference's minimap2 command when `minimap2` is given; otherwise `path`/Isoforms.aligned.out.sam
    must already exist."""
    sam = os.path.join(path, "Isoforms.aligned.out.sam")
    fsam = os.path.join(path, "Isoforms.aligned.out.filtered.sam")
    pslf = os.path.join(path, "Isoforms.aligned.out.psl")
    clean = os.path.join(path, "Isoforms.aligned.out.clean.psl")
    if minimap2:
        with open(sam, "w") as out:
            subprocess.run([minimap2, "-G", "400k", "-uf", "--secondary=no", "-ax", "splice:hq", "-t", str(threads),
                            genome_fasta, isoform_fasta], stdout=out, check=True)
    if not os.path.exists(sam):
        raise FileNotFoundError(f"{sam} (consensus alignments; pass an aligner or provide the SAM)")
    filter_sam(sam, fsam)
    psl.sam_to_psl(fsam, pslf, mando=False, threads=threads)
    psl.clean_psl(pslf, clean, False)
    out_fa = os.path.join(path, "Isoforms.filtered.fasta")
    out_psl = os.path.join(path, "Isoforms.filtered.clean.psl")
    wl = os.path.join(path, "polyAWhiteList.bed")
    n = filter_isoforms(params, isoform_fasta, genome_fasta, clean, wl, out_fa, out_psl,
                        os.path.join(path, "filter_reasons.txt"), device=device)
    psl_to_gtf(out_psl, os.path.join(path, "Isoforms.filtered.clean.gtf"))
    return n


def quantify(folder: str, fasta_files: list[str], device="auto") -> None:
    """assignReadsToIsoforms.py -m folder -f files: Isoforms.filtered.clean.quant / .tpm in folder.
    device: a GPU ordinal (the joins on the GPU, mando_quantify_device), None (host C++, mando_quantify) or
    "auto" (GPU 0 when one is visible)."""
    arr = (ctypes.c_char_p * len(fasta_files))(*[f.encode() for f in fasta_files])
    paths = [os.path.join(folder, f).encode() for f in ("reads2isoforms.txt", "Isoforms.filtered.clean.psl",
                                                          "Isoforms.filtered.clean.quant", "Isoforms.filtered.clean.tpm")]
    dev = _device(device)
    lib = _lib.load()
    if dev is None:
        _lib.check(lib.mando_quantify(arr, len(fasta_files), *paths))
    else:
        _lib.check(lib.mando_quantify_device(_lib.context(int(dev), slot=4).handle, arr, len(fasta_files), *paths))
