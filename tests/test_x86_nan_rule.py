"""CPU: the oracle's floating-point NaN rule is the x86 SSE hardware's.

The reference's float kernels (op.cpp:42-64 Sum/Prod, 289-300 complex) run as
scalar SSE instructions on x86-64.  IEEE 754 leaves a NaN result's payload
open, so the oracle states the platform rule explicitly (oracle/msx_oracle.c
X86_OP: first operand's NaN quieted, else the second's, else the default NaN
0xFFC00000 / 0xFFF8...) and the GPU kernels apply the same rule
(msx_dev_ops.h), checked bit for bit against the oracle on the GPU
(test_gpu_local.py).  A rule shared by kernel and oracle could still be wrong
in both; this test pins it to the silicon: tests/c/x86_sse_probe.c executes
addss/subss/mulss/addsd/subsd/mulsd (and maxss/minss/maxsd/minsd, whose
definition is the Windows max/min macro of op.cpp:26,38) with op.cpp's
operand order fixed by inline assembly, and every special-value pair (signed quiet and signalling
NaNs with payloads, infinities, zeros, denormals, finite values) must give
the oracle's bits.  What stays unpinned: the operand order MSVC emitted for
the commutative `+`/`*`."""
import ctypes
import itertools
import os
import platform
import subprocess

import numpy as np
import pytest

import msx
import oracle

C = msx.C
SRC = os.path.join(msx.REPO_ROOT, "tests", "c", "x86_sse_probe.c")

F32 = [0x7FC00000, 0xFFC00000, 0x7FC12345, 0xFFC54321, 0x7F800001, 0xFF812345, 0x7FBFFFFF,
       0x7F800000, 0xFF800000, 0x00000000, 0x80000000, 0x00000001, 0x807FFFFF, 0x3F800000,
       0xBF800000, 0x7F7FFFFF, 0x40490FDB, 0xC2F6E979]
F64 = [0x7FF8000000000000, 0xFFF8000000000000, 0x7FF8DEADBEEF0001, 0xFFF80000CAFE0000,
       0x7FF0000000000001, 0xFFF0123456789ABC, 0x7FF7FFFFFFFFFFFF, 0x7FF0000000000000,
       0xFFF0000000000000, 0x0000000000000000, 0x8000000000000000, 0x0000000000000001,
       0x800FFFFFFFFFFFFF, 0x3FF0000000000000, 0xBFF0000000000000, 0x7FEFFFFFFFFFFFFF,
       0x400921FB54442D18, 0xC05EDD2F1A9FBE77]


@pytest.fixture(scope="module")
def sse(tmp_path_factory):
    if platform.machine() not in ("x86_64", "AMD64"):
        pytest.skip("x86-64 host needed")
    so = str(tmp_path_factory.mktemp("sse") / "libx86sse.so")
    subprocess.run(["gcc", "-O2", "-shared", "-fPIC", "-o", so, SRC], check=True)
    L = ctypes.CDLL(so)
    for f in ("sse_f32", "sse_f64"):
        getattr(L, f).argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]
    for f in ("sse_c32_prod", "sse_c64_prod"):
        getattr(L, f).argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]
    return L


def _pairs(vals, udt):
    x, y = zip(*itertools.product(vals, vals))
    return np.array(x, udt), np.array(y, udt)


OPNUM = {"MPI_SUM": 0, "MPI_PROD": 1, "MPI_MAX": 2, "MPI_MIN": 3}


@pytest.mark.parametrize("op", list(OPNUM))
@pytest.mark.parametrize("width", [32, 64])
def test_real_ops_nan_payloads_match_sse(sse, op, width):
    vals, udt, fdt = (F32, np.uint32, np.float32) if width == 32 else (F64, np.uint64, np.float64)
    inout_bits, in_bits = _pairs(vals, udt)          # every (inout, in) pair, both orders
    dt = C.MPI_FLOAT if width == 32 else C.MPI_DOUBLE
    want = inout_bits.copy()
    fn = sse.sse_f32 if width == 32 else sse.sse_f64
    fn(OPNUM[op], in_bits.ctypes.data, want.ctypes.data, want.size)
    got = inout_bits.copy().view(fdt)
    assert oracle.reduce_local(getattr(C, op), dt, in_bits.view(fdt), got) == 0
    bad = np.nonzero(got.view(udt) != want)[0]
    assert bad.size == 0, [(hex(inout_bits[i]), hex(in_bits[i]), hex(got.view(udt)[i]), hex(want[i]))
                           for i in bad[:8]]
    # the table really exercises the rule: NaN results from NaN operands and
    # default NaNs from invalid operations on numbers (MAX/MIN: NaN in `in`)
    isnan = (want & (0x7F800000 if width == 32 else 0x7FF0000000000000)) == \
        (0x7F800000 if width == 32 else 0x7FF0000000000000)
    assert isnan.sum() > len(vals) * (6 if op in ("MPI_MAX", "MPI_MIN") else 8)


@pytest.mark.parametrize("width", [32, 64])
def test_complex_prod_nan_payloads_match_sse(sse, width):
    vals, udt, cdt = (F32, np.uint32, np.complex64) if width == 32 else (F64, np.uint64, np.complex128)
    rng = np.random.default_rng(width)
    n = 20000
    inout_bits = np.array(vals, udt)[rng.integers(0, len(vals), 2 * n)]
    in_bits = np.array(vals, udt)[rng.integers(0, len(vals), 2 * n)]
    want = inout_bits.copy()
    (sse.sse_c32_prod if width == 32 else sse.sse_c64_prod)(in_bits.ctypes.data, want.ctypes.data, n)
    dt = C.MPI_C_FLOAT_COMPLEX if width == 32 else C.MPI_C_DOUBLE_COMPLEX
    got = inout_bits.copy().view(cdt)
    assert oracle.reduce_local(C.MPI_PROD, dt, in_bits.view(cdt), got) == 0
    bad = np.nonzero(got.view(udt) != want)[0]
    assert bad.size == 0, [(i, hex(got.view(udt)[i]), hex(want[i])) for i in bad[:8]]
