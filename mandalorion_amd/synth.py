"""Synthetic R2C2 / PacBio-shaped read groups and loci (no network: the benchmark's data source).

Error model: R2C2 ~1% substitutions, 0.5% insertions, 0.5% deletions with indels
twice as likely inside homopolymers; PacBio HiFi-like 0.1% total.  Default data seed 20250117.
"""
from __future__ import annotations

import numpy as np

BASES = np.frombuffer(b"ACGT", dtype=np.uint8)
COMP = bytes.maketrans(b"ACGTNacgtn", b"TGCANtgcan")
DATA_SEED = 20250117

R2C2 = dict(sub=0.010, ins=0.005, dele=0.005)
PACBIO = dict(sub=0.0005, ins=0.00025, dele=0.00025)


def revcomp(s: str) -> str:
    return s.encode().translate(COMP)[::-1].decode()


def random_template(rng: np.random.Generator, length: int) -> np.ndarray:
    return BASES[rng.integers(0, 4, size=length)]


def _homopolymer_mask(t: np.ndarray) -> np.ndarray:
    hp = np.zeros(len(t), dtype=bool)
    if len(t) > 1:
        same = t[1:] == t[:-1]
        hp[1:] |= same
        hp[:-1] |= same
    return hp


def mutate(rng: np.random.Generator, t: np.ndarray, sub: float, ins: float, dele: float) -> np.ndarray:
    """One noisy copy of template t (uint8 ASCII array)."""
    n = len(t)
    f = np.where(_homopolymer_mask(t), 2.0, 1.0)
    u = rng.random(n)
    pd = dele * f
    is_del = u < pd
    is_sub = (~is_del) & (u < pd + sub)
    out = t.copy()
    if is_sub.any():
        idx = np.searchsorted(BASES, out[is_sub])
        out[is_sub] = BASES[(idx + rng.integers(1, 4, size=int(is_sub.sum()))) % 4]
    is_ins = rng.random(n) < ins * f
    keep = ~is_del
    if is_ins.any():
        # insertion after position i: homopolymer extension half the time, random base otherwise
        ins_base = np.where(rng.random(n) < 0.5, t, BASES[rng.integers(0, 4, size=n)])
        ins_base = ins_base[is_ins]
        pieces_idx = np.nonzero(is_ins)[0]
        body = out.copy()
        body_keep = keep
        # assemble: kept base (if any) followed by inserted base
        counts = body_keep.astype(np.int64) + is_ins.astype(np.int64)
        res = np.empty(int(counts.sum()), dtype=np.uint8)
        starts = np.concatenate([[0], np.cumsum(counts)[:-1]])
        kpos = starts[body_keep]
        res[kpos] = body[body_keep]
        ipos = starts[pieces_idx] + body_keep[pieces_idx].astype(np.int64)
        res[ipos] = ins_base
        return res
    return out[keep]


def read_group(rng: np.random.Generator, length: int, depth: int, model: dict = R2C2):
    """(template, reads) for one isoform: depth noisy copies of a random template of `length`."""
    t = random_template(rng, length)
    reads = [mutate(rng, t, **model).tobytes().decode() for _ in range(depth)]
    return t.tobytes().decode(), reads


def read_groups(n_groups: int, length: int | tuple[int, int], depth: int | tuple[int, int],
                seed: int = DATA_SEED, model: dict = R2C2):
    """n_groups groups; length/depth either fixed or an inclusive (lo, hi) uniform range."""
    rng = np.random.default_rng(seed)
    templates, groups = [], []
    for _ in range(n_groups):
        L = length if isinstance(length, int) else int(rng.integers(length[0], length[1] + 1))
        d = depth if isinstance(depth, int) else int(rng.integers(depth[0], depth[1] + 1))
        t, rs = read_group(rng, L, d, model)
        templates.append(t)
        groups.append(rs)
    return templates, groups


# ---------------------------------------------------------------------------------------------
# fast multithreaded generator (libmando_synth.so) for benchmark-scale data
# ---------------------------------------------------------------------------------------------
def _synth_lib():
    import ctypes
    import os

    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib", "libmando_synth.so")
    lib = ctypes.CDLL(path)
    P = ctypes.c_void_p
    lib.mando_synth_groups.argtypes = [ctypes.c_uint64, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32,
                                       ctypes.c_int32, ctypes.c_int32, ctypes.c_double, ctypes.c_double,
                                       ctypes.c_double, P, P, P, P, P, P, ctypes.c_int]
    lib.mando_synth_free.argtypes = [P]
    return lib


def fast_groups(n_groups: int, length: tuple[int, int], depth: tuple[int, int], seed: int = DATA_SEED,
                model: dict = R2C2, threads: int = 0, with_templates: bool = False):
    """Packed groups: (seqs uint8 array, seq_off int64, grp_off int64[, templates list])."""
    import ctypes

    lib = _synth_lib()
    out = ctypes.c_void_p()
    so = ctypes.c_void_p()
    nr = ctypes.c_int64()
    go = ctypes.c_void_p()
    tp = ctypes.c_void_p()
    to = ctypes.c_void_p()
    rc = lib.mando_synth_groups(seed, n_groups, length[0], length[1], depth[0], depth[1],
                                model["sub"], model["ins"], model["dele"], ctypes.byref(out),
                                ctypes.byref(so), ctypes.byref(nr), ctypes.byref(go),
                                ctypes.byref(tp) if with_templates else None,
                                ctypes.byref(to) if with_templates else None, threads)
    if rc != 0:
        raise RuntimeError(f"mando_synth_groups failed: {rc}")
    n = nr.value
    seq_off = np.ctypeslib.as_array(ctypes.cast(so, ctypes.POINTER(ctypes.c_int64)), shape=(n + 1,)).copy()
    grp_off = np.ctypeslib.as_array(ctypes.cast(go, ctypes.POINTER(ctypes.c_int64)), shape=(n_groups + 1,)).copy()
    total = int(seq_off[-1])
    seqs = np.ctypeslib.as_array(ctypes.cast(out, ctypes.POINTER(ctypes.c_uint8)), shape=(max(total, 1),)).copy()
    templates = None
    if with_templates:
        toff = np.ctypeslib.as_array(ctypes.cast(to, ctypes.POINTER(ctypes.c_int64)), shape=(n_groups + 1,)).copy()
        traw = ctypes.string_at(tp, int(toff[-1]))
        templates = [traw[toff[i]:toff[i + 1]].decode() for i in range(n_groups)]
        lib.mando_synth_free(tp)
        lib.mando_synth_free(to)
    for p in (out, so, go):
        lib.mando_synth_free(p)
    return (seqs, seq_off, grp_off, templates) if with_templates else (seqs, seq_off, grp_off)


def unpack_groups(seqs: np.ndarray, seq_off: np.ndarray, grp_off: np.ndarray, groups=None):
    """Packed -> list of lists of str (optionally only the listed group indices)."""
    raw = seqs.tobytes()
    idx = range(len(grp_off) - 1) if groups is None else groups
    return [[raw[seq_off[r]:seq_off[r + 1]].decode() for r in range(grp_off[g], grp_off[g + 1])] for g in idx]


def write_loci(tmp_ss: str, n_loci: int, reads: tuple[int, int] = (50, 50), exons: tuple[int, int] = (5, 12),
               exon_len: tuple[int, int] = (150, 400), intron_len: tuple[int, int] = (300, 3000),
               isoforms: tuple[int, int] = (1, 3), seed: int = DATA_SEED, model: dict = R2C2,
               threads: int = 0, pacbio_frac: float = 0.0, rev_frac: float = 0.0) -> int:
    """Benchmark-scale locus PSL files (libmando_synth mando_synth_loci, same format as simdata.py) into
    tmp_ss; returns the number of PSL records written.  pacbio_frac of the reads use the PacBio error
    rates (config 4's mix); rev_frac of them are '-' strand records (reverse-complemented read)."""
    import ctypes
    import os

    lib = _synth_lib()
    lib.mando_synth_loci.restype = ctypes.c_int64
    lib.mando_synth_loci.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_int64] + [ctypes.c_int32] * 10 + \
        [ctypes.c_double] * 8 + [ctypes.c_int]
    os.makedirs(tmp_ss, exist_ok=True)
    n = lib.mando_synth_loci(tmp_ss.encode(), seed, n_loci, reads[0], reads[1], exons[0], exons[1], exon_len[0],
                             exon_len[1], intron_len[0], intron_len[1], isoforms[0], isoforms[1], model["sub"],
                             model["ins"], model["dele"], pacbio_frac, PACBIO["sub"], PACBIO["ins"],
                             PACBIO["dele"], rev_frac, threads)
    if n < 0:
        raise RuntimeError(f"mando_synth_loci failed: {n}")
    return int(n)
