"""msx — Python binding of libmsmpi_mi355x.so (the MI355X MS-MPI reduction path).

Thin ctypes layer over the C ABI declared in include/mpi.h and include/msx.h,
used by the tests, bench.py and __graft_entry__.py.  The library is the
product; nothing here computes a reduction.  If the shared library is missing
the import of `lib()` raises: there is no Python or CPU fallback.
"""
from __future__ import annotations

import ctypes
import os
import re
from types import SimpleNamespace

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(_HERE)                      # microsoft-mpi_amd/
REPO_ROOT = os.path.dirname(PKG_ROOT)
LIB_PATH = os.path.join(PKG_ROOT, "lib", "libmsmpi_mi355x.so")
INCLUDE_DIR = os.path.join(REPO_ROOT, "include")

_lib = None


def _parse_header_constants(path):
    """#define NAME value / ((T)0x...) from include/mpi.h -> dict (ints only)."""
    out = {}
    pat = re.compile(r"^#define\s+(MPI_\w+)\s+(.+?)\s*(?:/\*.*)?$")
    enum = re.compile(r"^(MPI_\w+)\s*=\s*(\d+),?$")
    with open(path) as f:
        for line in f:
            e = enum.match(line.strip())
            if e:
                out[e.group(1)] = int(e.group(2))
                continue
            m = pat.match(line.strip())
            if not m:
                continue
            name, val = m.group(1), m.group(2).strip()
            val = re.sub(r"\(\((?:MPI_\w+|void\*|MPI_Status\*)\)(?:\(MPI_Aint\))?(.+?)\)$", r"\1", val)
            val = val.strip("() ")
            try:
                out[name] = int(val, 0)
            except ValueError:
                if val in out:
                    out[name] = out[val]
    return out


C = SimpleNamespace(**_parse_header_constants(os.path.join(INCLUDE_DIR, "mpi.h")))


def _signed32(v):
    v &= 0xFFFFFFFF
    return v - (1 << 32) if v & 0x80000000 else v


# all handle values as C ints (MPI_Datatype / MPI_Op are `int`)
for _k, _v in list(vars(C).items()):
    setattr(C, _k, _signed32(_v))


def lib():
    """Load the HIP library (raises OSError if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise OSError(f"{LIB_PATH} missing: run `make -C microsoft-mpi_amd` (or __graft_entry__.build())")
    L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    i, p, i64 = ctypes.c_int, ctypes.c_void_p, ctypes.c_int64
    sig = {
        "MPI_Init": (i, [p, p]),
        "MPI_Finalize": (i, []),
        "MPI_Initialized": (i, [ctypes.POINTER(i)]),
        "MPI_Finalized": (i, [ctypes.POINTER(i)]),
        "MPI_Comm_rank": (i, [i, ctypes.POINTER(i)]),
        "MPI_Comm_size": (i, [i, ctypes.POINTER(i)]),
        "MPI_Barrier": (i, [i]),
        "MPI_Comm_split": (i, [i, i, i, ctypes.POINTER(i)]),
        "MPI_Comm_dup": (i, [i, ctypes.POINTER(i)]),
        "MPI_Comm_free": (i, [ctypes.POINTER(i)]),
        "MPI_Comm_set_errhandler": (i, [i, i]),
        "MPI_Error_class": (i, [i, ctypes.POINTER(i)]),
        "MPI_Type_size": (i, [i, ctypes.POINTER(i)]),
        "MPI_Op_create": (i, [p, i, ctypes.POINTER(i)]),
        "MPI_Op_free": (i, [ctypes.POINTER(i)]),
        "MPI_Op_commutative": (i, [i, ctypes.POINTER(i)]),
        "MPI_Reduce_local": (i, [p, p, i, i, i]),
        "MPI_Reduce": (i, [p, p, i, i, i, i, i]),
        "MPI_Allreduce": (i, [p, p, i, i, i, i]),
        "MPI_Reduce_scatter": (i, [p, p, p, i, i, i]),
        "MPI_Reduce_scatter_block": (i, [p, p, i, i, i, i]),
        "MPI_Iallreduce": (i, [p, p, i, i, i, i, ctypes.POINTER(i)]),
        "MPI_Ireduce": (i, [p, p, i, i, i, i, i, ctypes.POINTER(i)]),
        "MPI_Ireduce_scatter_block": (i, [p, p, i, i, i, i, ctypes.POINTER(i)]),
        "MPI_Ireduce_scatter": (i, [p, p, p, i, i, i, ctypes.POINTER(i)]),
        "MPI_Waitall": (i, [i, ctypes.POINTER(i), p]),
        "MPI_Scan": (i, [p, p, i, i, i, i]),
        "MPI_Exscan": (i, [p, p, i, i, i, i]),
        "MPI_Iscan": (i, [p, p, i, i, i, i, ctypes.POINTER(i)]),
        "MPI_Iexscan": (i, [p, p, i, i, i, i, ctypes.POINTER(i)]),
        "MPI_Win_create": (i, [p, i64, i, i, i, ctypes.POINTER(i)]),
        "MPI_Win_allocate": (i, [i64, i, i, i, p, ctypes.POINTER(i)]),
        "MPI_Alloc_mem": (i, [i64, i, p]),
        "MPI_Free_mem": (i, [p]),
        "MPI_Win_free": (i, [ctypes.POINTER(i)]),
        "MPI_Win_fence": (i, [i, i]),
        "MPI_Win_lock": (i, [i, i, i, i]),
        "MPI_Win_unlock": (i, [i, i]),
        "MPI_Win_lock_all": (i, [i, i]),
        "MPI_Win_unlock_all": (i, [i]),
        "MPI_Win_flush": (i, [i, i]),
        "MPI_Win_flush_all": (i, [i]),
        "MPI_Win_flush_local": (i, [i, i]),
        "MPI_Win_flush_local_all": (i, [i]),
        "MPI_Win_sync": (i, [i]),
        "MPI_Win_set_errhandler": (i, [i, i]),
        "MPI_Win_get_errhandler": (i, [i, ctypes.POINTER(i)]),
        "MPI_Put": (i, [p, i, i, i, i64, i, i, i]),
        "MPI_Get": (i, [p, i, i, i, i64, i, i, i]),
        "MPI_Accumulate": (i, [p, i, i, i, i64, i, i, i, i]),
        "MPI_Get_accumulate": (i, [p, i, i, p, i, i, i, i64, i, i, i, i]),
        "MPI_Fetch_and_op": (i, [p, p, i, i, i64, i, i]),
        "MPI_Compare_and_swap": (i, [p, p, p, i, i, i64, i]),
        # derived datatypes + pack (msx_dtype_api.cpp); arrays / outputs as void*
        "MPI_Type_contiguous": (i, [i, i, p]),
        "MPI_Type_vector": (i, [i, i, i, i, p]),
        "MPI_Type_create_hvector": (i, [i, i, i64, i, p]),
        "MPI_Type_hvector": (i, [i, i, i64, i, p]),
        "MPI_Type_indexed": (i, [i, p, p, i, p]),
        "MPI_Type_create_hindexed": (i, [i, p, p, i, p]),
        "MPI_Type_hindexed": (i, [i, p, p, i, p]),
        "MPI_Type_create_indexed_block": (i, [i, i, p, i, p]),
        "MPI_Type_create_hindexed_block": (i, [i, i, p, i, p]),
        "MPI_Type_create_struct": (i, [i, p, p, p, p]),
        "MPI_Type_struct": (i, [i, p, p, p, p]),
        "MPI_Type_create_subarray": (i, [i, p, p, p, i, i, p]),
        "MPI_Type_create_resized": (i, [i, i64, i64, p]),
        "MPI_Type_create_darray": (i, [i, i, i, p, p, p, p, i, i, p]),
        "MPI_Type_dup": (i, [i, p]),
        "MPI_Type_commit": (i, [p]),
        "MPI_Type_free": (i, [p]),
        "MPI_Type_size_x": (i, [i, p]),
        "MPI_Type_get_extent": (i, [i, p, p]),
        "MPI_Type_get_extent_x": (i, [i, p, p]),
        "MPI_Type_get_true_extent": (i, [i, p, p]),
        "MPI_Type_get_true_extent_x": (i, [i, p, p]),
        "MPI_Type_extent": (i, [i, p]),
        "MPI_Type_lb": (i, [i, p]),
        "MPI_Type_ub": (i, [i, p]),
        "MPI_Type_get_envelope": (i, [i, p, p, p, p]),
        "MPI_Type_get_contents": (i, [i, i, i, i, p, p, p]),
        "MPI_Get_address": (i, [p, p]),
        "MPI_Pack": (i, [p, i, i, p, i, p, i]),
        "MPI_Unpack": (i, [p, i, p, p, i, i, i]),
        "MPI_Pack_size": (i, [i, i, i, p]),
        "msx_engine_transport": (ctypes.c_char_p, []),
        "msx_engine_stats": (i, [ctypes.POINTER(ctypes.c_double), i, i]),
        "msx_engine_gpu_shared": (i, []),
        "msx_peer_write_bandwidth": (i, [i64, i, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(i64)]),
        "MPI_Wait": (i, [ctypes.POINTER(i), p]),
        "MPI_Test": (i, [ctypes.POINTER(i), ctypes.POINTER(i), p]),
        "MPI_Wtime": (ctypes.c_double, []),
        "msx_version": (ctypes.c_char_p, []),
        "msx_device_count": (i, []),
        "msx_last_error": (ctypes.c_char_p, []),
        "msx_op_check": (i, [i, i]),
        "msx_operands_on_device": (i, [p, p]),
        "msx_schedule_two_step": (i64, [i, i64, i, i, ctypes.POINTER(i64), ctypes.POINTER(i64), i64]),
        "msx_reduce_local_multi": (i, [p, p, i64, i, i, i]),
        "msx_reduce_tree_spec_dev": (i, [ctypes.POINTER(p), i, ctypes.c_uint, i, i, p, i64, i, i, p]),
        "msx_type_size": (i, [i]),
        "msx_reduce_local_dev": (i, [p, p, i64, i, i, p]),
        "msx_pack_dev": (i, [p, i64, i, p, p]),
        "msx_unpack_dev": (i, [p, i64, i, p, p]),
        "msx_reduce_tree_dev": (i, [ctypes.POINTER(p), i, p, i64, i, i, p]),
        "msx_tune_pack": (i, [i]),
        "msx_copy_dev": (i, [p, p, i64, p]),
        "msx_set_staging_chunk": (i, [i64]),
        "msx_set_host_mode": (i, [i]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def exported_symbols():
    """Names the C headers declare (MPI_*/PMPI_*/msx_* prototypes)."""
    names = set()
    for h in ("mpi.h", "msx.h"):
        with open(os.path.join(INCLUDE_DIR, h)) as f:
            txt = f.read()
        names.update(re.findall(
            r"(?:MPI_METHOD|double MPIAPI|const char\*|int|void|MPI_User_function\*)\s+((?:P?MPI|msx)_\w+)\s*\(", txt))
    return sorted(names)


def ptr(x):
    """Raw address of a torch tensor, numpy array, int or None."""
    if x is None:
        return None
    if isinstance(x, int):
        return x
    if hasattr(x, "data_ptr"):
        return x.data_ptr()
    if hasattr(x, "ctypes"):
        return x.ctypes.data
    raise TypeError(type(x))


def last_error():
    return lib().msx_last_error().decode()


def init(errors_return=True):
    """MPI_Init once; by default switch COMM_WORLD to MPI_ERRORS_RETURN."""
    L = lib()
    flag = ctypes.c_int(0)
    L.MPI_Initialized(ctypes.byref(flag))
    if not flag.value:
        rc = L.MPI_Init(None, None)
        if rc:
            raise RuntimeError(f"MPI_Init failed: {rc} {last_error()}")
    if errors_return:
        L.MPI_Comm_set_errhandler(C.MPI_COMM_WORLD, C.MPI_ERRORS_RETURN)
    return L


# element kinds per datatype, as the reference's CASE_MPI_* macros map them
# (mpid/op.cpp:343-536, LLP64); numpy dtype strings for test data.
LOC_DTYPES = {
    "ii": [("v", "<i4"), ("l", "<i4")],
    "fi": [("v", "<f4"), ("l", "<i4")],
    "si": {"names": ["v", "l"], "formats": ["<i2", "<i4"], "offsets": [0, 4], "itemsize": 8},
    "di": {"names": ["v", "l"], "formats": ["<f8", "<i4"], "offsets": [0, 8], "itemsize": 16},
    "ff": [("v", "<f4"), ("l", "<f4")],
    "dd": [("v", "<f8"), ("l", "<f8")],
}
