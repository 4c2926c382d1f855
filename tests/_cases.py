"""Test-case tables: every predefined datatype, its element class (as the
reference's CASE_MPI_* macros map it, mpid/op.cpp:343-536, LLP64), and seeded
input generators that hit the edge values the reference semantics pin
(integer wrap, NaN / +-0 for MAX/MIN, ties for MAXLOC/MINLOC, zeros for the
logical ops, denormals)."""
import numpy as np

import msx

C = msx.C

# datatype name -> element class
KIND = {
    "MPI_INT": "i4", "MPI_LONG": "i4", "MPI_SHORT": "i2", "MPI_UNSIGNED_SHORT": "u2",
    "MPI_UNSIGNED": "u4", "MPI_UNSIGNED_LONG": "u4", "MPI_LONG_LONG": "i8",
    "MPI_UNSIGNED_LONG_LONG": "u8", "MPI_SIGNED_CHAR": "i1", "MPI_UNSIGNED_CHAR": "u1",
    "MPI_INT8_T": "i1", "MPI_INT16_T": "i2", "MPI_INT32_T": "i4", "MPI_INT64_T": "i8",
    "MPI_UINT8_T": "u1", "MPI_UINT16_T": "u2", "MPI_UINT32_T": "u4", "MPI_UINT64_T": "u8",
    "MPI_INTEGER": "i4", "MPI_AINT": "i8", "MPI_OFFSET": "i8", "MPI_INTEGER1": "i1",
    "MPI_INTEGER2": "i2", "MPI_INTEGER4": "i4", "MPI_INTEGER8": "i8",
    "MPI_FLOAT": "f4", "MPI_REAL": "f4", "MPI_REAL4": "f4", "MPI_DOUBLE": "f8",
    "MPI_DOUBLE_PRECISION": "f8", "MPI_REAL8": "f8", "MPI_LONG_DOUBLE": "f8",
    "MPI_COMPLEX8": "c8", "MPI_COMPLEX": "c8", "MPI_C_COMPLEX": "c8", "MPI_C_FLOAT_COMPLEX": "c8",
    "MPI_COMPLEX16": "c16", "MPI_DOUBLE_COMPLEX": "c16", "MPI_C_DOUBLE_COMPLEX": "c16",
    "MPI_C_LONG_DOUBLE_COMPLEX": "c16",
    "MPI_LOGICAL": "i4", "MPI_C_BOOL": "b1", "MPI_BYTE": "u1", "MPI_CHAR": "i1", "MPI_CHARACTER": "i1",
    "MPI_2INT": "ii", "MPI_2INTEGER": "ii", "MPI_LONG_INT": "ii", "MPI_FLOAT_INT": "fi",
    "MPI_SHORT_INT": "si", "MPI_DOUBLE_INT": "di", "MPI_LONG_DOUBLE_INT": "di",
    "MPI_2REAL": "ff", "MPI_2DOUBLE_PRECISION": "dd",
}
# predefined but never reducible with builtin ops
NON_REDUCIBLE = ["MPI_WCHAR", "MPI_PACKED", "MPI_LB", "MPI_UB", "MPI_COUNT", "MPI_2COMPLEX",
                 "MPI_2DOUBLE_COMPLEX"]

OPS = ["MPI_MAX", "MPI_MIN", "MPI_SUM", "MPI_PROD", "MPI_LAND", "MPI_BAND", "MPI_LOR",
       "MPI_BOR", "MPI_LXOR", "MPI_BXOR", "MPI_MINLOC", "MPI_MAXLOC"]


def h(name):
    return getattr(C, name)


def np_dtype(kind):
    if kind in msx.LOC_DTYPES:
        return np.dtype(msx.LOC_DTYPES[kind])
    return np.dtype({"b1": "u1", "c8": "c8", "c16": "c16"}.get(kind, kind))


def itemsize(kind):
    return np_dtype(kind).itemsize


def legal_pairs(oracle_mod):
    out = []
    for op in OPS:
        for dt in KIND:
            if oracle_mod.op_check(h(op), h(dt)) == 0:
                out.append((op, dt))
    return out


def _float_edges(ft):
    info = np.finfo(ft)
    return np.array([0.0, -0.0, np.nan, np.inf, -np.inf, 1.0, -1.0, info.tiny / 4, -info.tiny / 2,
                     info.max, -info.max, 1.5, 1.5], dtype=ft)


def gen(kind, op, n, rng):
    """Random buffer of n elements of `kind`, with edge values mixed in."""
    if n == 0:
        return np.zeros(0, dtype=np_dtype(kind))
    logical = op in ("MPI_LAND", "MPI_LOR", "MPI_LXOR")
    if kind in ("i1", "u1", "i2", "u2", "i4", "u4", "i8", "u8"):
        a = rng.integers(0, 256, size=n * np.dtype(kind).itemsize, dtype=np.uint8).view(kind).copy()
        if op in ("MPI_MAX", "MPI_MIN"):
            a[rng.random(n) < 0.2] = 7          # ties
        if logical:
            a[rng.random(n) < 0.4] = 0
        if op == "MPI_PROD":
            a[rng.random(n) < 0.1] = 0
        return a
    if kind == "b1":
        return (rng.random(n) < 0.5).astype(np.uint8)
    if kind in ("f4", "f8"):
        a = rng.uniform(-4, 4, size=n).astype(kind)
        m = rng.random(n)
        e = _float_edges(kind)
        sel = m < 0.25
        a[sel] = e[rng.integers(0, len(e), size=int(sel.sum()))]
        if logical:
            a[rng.random(n) < 0.3] = 0.0
        return a
    if kind in ("c8", "c16"):
        ft = "f4" if kind == "c8" else "f8"
        re = rng.uniform(-2, 2, size=n).astype(ft)
        im = rng.uniform(-2, 2, size=n).astype(ft)
        a = np.empty(n, dtype=kind)
        a.real, a.imag = re, im
        return a
    # value/location pairs: small value set for ties, NaN for float values
    a = np.zeros(n, dtype=np_dtype(kind))
    vals = rng.integers(-3, 4, size=n)
    if kind in ("fi", "ff", "di", "dd"):
        v = vals.astype(np.float64)
        v[rng.random(n) < 0.05] = np.nan
        a["v"] = v
    else:
        a["v"] = vals
    a["l"] = rng.integers(-50, 50, size=n)
    return a


def bytes_equal(x, y):
    return np.array_equal(np.frombuffer(x.tobytes(), np.uint8), np.frombuffer(y.tobytes(), np.uint8))


def loc_payload_equal(x, y):
    """Compare value+location fields bitwise (padding bytes excluded)."""
    return (np.array_equal(x["v"].view(np.uint8), y["v"].view(np.uint8))
            and np.array_equal(x["l"].view(np.uint8), y["l"].view(np.uint8)))
