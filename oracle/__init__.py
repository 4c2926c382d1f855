"""ORACLE — test infrastructure only.

ctypes wrapper around oracle/liboracle.so, the plain-C restatement of MS-MPI's
MPI_Op kernels (msx_oracle.c) and reduction schedules (msx_oracle_sched.c).
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this package; the product library never links or calls it.

Parity UNPINNED in this task's terms: the known-answer vectors
in tests/golden/survey_kat.json were recorded from op.cpp built with a probe
shim, which does not count as a reference build; x86 silicon anchors the
float / NaN rules (tests/test_x86_nan_rule.py).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        build()
    L = ctypes.CDLL(LIB_PATH)
    i, p, i64 = ctypes.c_int, ctypes.c_void_p, ctypes.c_int64
    L.oracle_kind_of.restype = i
    L.oracle_kind_of.argtypes = [i]
    L.oracle_kind_size.restype = i
    L.oracle_kind_size.argtypes = [i]
    L.oracle_op_check.restype = i
    L.oracle_op_check.argtypes = [i, i]
    L.oracle_reduce_local.restype = i
    L.oracle_reduce_local.argtypes = [i, i, p, p, i64]
    L.oracle_reduce_local_mt.restype = i
    L.oracle_reduce_local_mt.argtypes = [i, i, p, p, i64, i]
    L.oracle_allreduce.restype = i
    L.oracle_allreduce.argtypes = [i, i, i, i64, ctypes.POINTER(p), ctypes.POINTER(p)]
    L.oracle_reduce.restype = i
    L.oracle_reduce.argtypes = [i, i, i, i, i64, ctypes.POINTER(p), p]
    L.oracle_scan.restype = i
    L.oracle_scan.argtypes = [i, i, i, i64, i, ctypes.POINTER(p), ctypes.POINTER(p)]
    L.oracle_type_size.restype = i
    L.oracle_type_size.argtypes = [i]
    L.oracle_iallreduce.restype = i
    L.oracle_iallreduce.argtypes = [i, i, i, i64, ctypes.POINTER(p), ctypes.POINTER(p)]
    L.oracle_ireduce.restype = i
    L.oracle_ireduce.argtypes = [i, i, i, i, i64, ctypes.POINTER(p), p]
    L.oracle_reduce_scatter.restype = i
    L.oracle_reduce_scatter.argtypes = [i, i, i, ctypes.POINTER(i), ctypes.POINTER(p), ctypes.POINTER(p)]
    L.oracle_coll_threads.restype = i
    L.oracle_coll_threads.argtypes = [i, i, i, i, i64, i, ctypes.POINTER(ctypes.c_double)]
    _lib = L
    return L


def _addr(a):
    return a.ctypes.data


def reduce_local(op, dt, inbuf, inoutbuf, count=None, nthreads=1):
    """inoutbuf (numpy) = inoutbuf op inbuf, in place.  Returns op_errno."""
    n = count if count is not None else inoutbuf.size
    if nthreads > 1:
        return lib().oracle_reduce_local_mt(op, dt, _addr(inbuf), _addr(inoutbuf), n, nthreads)
    return lib().oracle_reduce_local(op, dt, _addr(inbuf), _addr(inoutbuf), n)


def op_check(op, dt):
    return lib().oracle_op_check(op, dt)


def kind_size(dt):
    return lib().oracle_kind_size(lib().oracle_kind_of(dt))


def allreduce(op, dt, sendbufs, recvbufs):
    p = len(sendbufs)
    S = (ctypes.c_void_p * p)(*[_addr(b) for b in sendbufs])
    R = (ctypes.c_void_p * p)(*[_addr(b) for b in recvbufs])
    return lib().oracle_allreduce(op, dt, p, sendbufs[0].size, S, R)


def type_size(dt):
    """MPI_Type_size of a reducible predefined type (12 for MPI_DOUBLE_INT)."""
    return lib().oracle_type_size(dt)


def iallreduce(op, dt, sendbufs, recvbufs):
    """MPI_Iallreduce's NBC task list (extent gate, reduce.cpp:4699-4982)."""
    p = len(sendbufs)
    S = (ctypes.c_void_p * p)(*[_addr(b) for b in sendbufs])
    R = (ctypes.c_void_p * p)(*[_addr(b) for b in recvbufs])
    return lib().oracle_iallreduce(op, dt, p, sendbufs[0].size, S, R)


def ireduce(op, dt, root, sendbufs, recvbuf):
    """MPI_Ireduce's NBC task list (extent gate, root-relative Rabenseifner,
    reduce.cpp:6005-6768)."""
    p = len(sendbufs)
    S = (ctypes.c_void_p * p)(*[_addr(b) for b in sendbufs])
    return lib().oracle_ireduce(op, dt, p, root, sendbufs[0].size, S, _addr(recvbuf))


def reduce_scatter(op, dt, recvcounts, sendbufs, recvbufs):
    p = len(sendbufs)
    S = (ctypes.c_void_p * p)(*[_addr(b) for b in sendbufs])
    R = (ctypes.c_void_p * p)(*[_addr(b) for b in recvbufs])
    C = (ctypes.c_int * p)(*recvcounts)
    return lib().oracle_reduce_scatter(op, dt, p, C, S, R)


def reduce(op, dt, root, sendbufs, recvbuf):
    p = len(sendbufs)
    S = (ctypes.c_void_p * p)(*[_addr(b) for b in sendbufs])
    return lib().oracle_reduce(op, dt, p, root, sendbufs[0].size, S, _addr(recvbuf))


def scan(op, dt, sendbufs, recvbufs, exclusive=False):
    p = len(sendbufs)
    S = (ctypes.c_void_p * p)(*[_addr(b) for b in sendbufs])
    R = (ctypes.c_void_p * p)(*[_addr(b) for b in recvbufs])
    return lib().oracle_scan(op, dt, p, sendbufs[0].size, 1 if exclusive else 0, S, R)


def coll_threads(which, op, dt, p, count, reps):
    """p threads as p ranks run the reference's collective step loop
    (msx_oracle_threads.c): which 0 = allreduce, 1 = reduce_scatter_block.
    Returns (rc, [seconds per call])."""
    t = (ctypes.c_double * reps)()
    rc = lib().oracle_coll_threads(which, op, dt, p, count, reps, t)
    return rc, list(t)
