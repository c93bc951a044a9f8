"""The C-ABI library loads and exports every symbol include/mando.h declares (no GPU needed)."""
import ctypes
import os
import re

import numpy as np
import pytest

from mandalorion_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    src = open(os.path.join(ROOT, "include", "mando.h")).read()
    return sorted(set(re.findall(r"^(?:const\s+)?[a-z0-9_]+\s*\*?\s*(mando_[a-z0-9_]+)\s*\(", src, re.M)))


def test_header_matches_export_list():
    assert header_symbols() == sorted(_lib.EXPORTED)


def test_library_exports_every_header_symbol():
    lib = _lib.load()
    missing = [s for s in header_symbols() if not hasattr(lib, s)]
    assert not missing, missing


def test_default_params_are_abpoa_M5():
    p = _lib.PoaParams.defaults()
    assert (p.match, p.mismatch, p.gap_open1, p.gap_ext1, p.gap_open2, p.gap_ext2) == (5, 4, 4, 2, 24, 1)
    assert p.band_b == 10 and abs(p.band_f - 0.01) < 1e-7 and p.seeding == 0
    assert (p.k, p.w, p.min_w) == (19, 10, 500)


def test_abi_version():
    assert _lib.load().mando_abi_version() == 1


def test_device_count_never_fails():
    assert _lib.device_count() >= 0


def test_ctx_create_fails_loudly_without_gpu():
    if _lib.device_count() > 0:
        return
    h = ctypes.c_void_p()
    rc = _lib.load().mando_ctx_create(0, ctypes.byref(h))
    assert rc == -7 and not h.value
    assert b"no HIP device" in _lib.load().mando_last_error()


def test_bad_arguments_rejected():
    lib = _lib.load()
    out = np.zeros(4, dtype=np.int64)
    ns = np.array([5], dtype=np.int64)
    ks = np.array([6], dtype=np.int64)  # k > n
    assert lib.mando_mt_permutation(0, ns.ctypes.data, ks.ctypes.data, 1, out.ctypes.data, 4) == -1
    assert lib.mando_poa_batch(None, None, None, None, None, 0, None, None, 0, None, None) == -1


@pytest.mark.gpu
def test_ctx_sets_blocking_sync():
    """mando_ctx_create puts the device's host waits on blocking sync (include/mando.h), and says so."""
    from mandalorion_amd import _lib

    c = _lib.context(0)
    assert c.lib.mando_ctx_blocking_sync(c.handle) == 1
