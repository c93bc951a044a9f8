"""mandalorion_amd — MI355X-native consensus core for Mandalorion's D module.

Hot path: per-isoform read orientation and partial-order-alignment consensus run as
HIP kernels for gfx950 behind the C-ABI in include/mando.h (libmando.so, bound with ctypes in
_lib.py).  The host side (defineIsoforms / Mando.py -M D) stays Python.
"""
__version__ = "0.1.0"
