"""msx.probe — ctypes binding of libmsx_probe.so, the bench-only measurement
kernels (microsoft-mpi_amd/probe/msx_probe.hip): HBM stream-mix probes and the
fp32 SUM combine body in other launch geometries.  Used by bench.py, the
scripts and the GPU tests that check the variants compute the same bits; the
product library libmsmpi_mi355x.so neither contains nor loads any of it.
"""
from __future__ import annotations

import ctypes
import os

from . import PKG_ROOT

PROBE_PATH = os.path.join(PKG_ROOT, "lib", "libmsx_probe.so")

# msxp_hbm modes
READ2, WRITE1, COPY, READ1, GAP_STORE, GAP_LOAD, COPY_DISPATCH_ORDER, COPY_XCD_RUNS = 0, 1, 2, 3, 6, 7, 9, 10

_lib = None


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(PROBE_PATH):
        raise RuntimeError(f"{PROBE_PATH} not built: run `make -C microsoft-mpi_amd` (or __graft_entry__.build())")
    L = ctypes.CDLL(PROBE_PATH)
    p, i, i64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
    for name, res, args in (("msxp_hbm", i, [i, p, p, i64, p]),
                            ("msxp_alloc", i, [i64, i, ctypes.POINTER(p)]),
                            ("msxp_free", i, [p]),
                            ("msxp_variant_count", i, []),
                            ("msxp_variant_name", ctypes.c_char_p, [i]),
                            ("msxp_variant_run", i, [i, p, p, i64, p]),
                            ("msxp_tree8", i, [ctypes.POINTER(p), p, i64, i, p]),
                            ("msxp_spin_mark", i, [i64, p, ctypes.c_uint, p])):
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def variants():
    """{name: index} of the fp32 SUM combine variants (index 0 = the product's
    default DRAM-regime body under its probe symbol)."""
    L = lib()
    return {L.msxp_variant_name(v).decode(): v for v in range(L.msxp_variant_count())}
