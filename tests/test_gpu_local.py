"""GPU parity: the HIP combine kernels vs the oracle, through the C ABI.

Every legal (op, datatype) pair of the reference (op.cpp:739-1883) runs on the
MI355X on seeded inputs with edge values (wrap, NaN, +-0, inf, denormals,
ties, zeros) and must match the oracle BIT-EXACTLY: each element is one IEEE
operation or one integer/logical/bitwise operation, exactly as in op.cpp, so
no tolerance applies (not even for floating point).  Also covered: ragged
sizes, unaligned and mutually misaligned pointers, host (pageable / pinned)
buffers through MPI_Reduce_local's staged path, the reference's known-answer
vectors, and a size-independent check at the benchmark size (256 MiB fp32).
"""
import ctypes
import json
import os
import zlib

import numpy as np
import pytest

import msx
import oracle
from _cases import KIND, OPS, gen, h, itemsize, legal_pairs, np_dtype

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

C = msx.C


@pytest.fixture(scope="module")
def L():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    lib = msx.init(errors_return=True)
    assert lib.msx_device_count() > 0
    return lib


def _dev(a, offset=0):
    """Copy numpy array bytes into a fresh device buffer at byte `offset`."""
    raw = np.frombuffer(a.tobytes(), np.uint8)
    t = torch.zeros(raw.size + offset + 64, dtype=torch.uint8, device="cuda")
    if raw.size:   # page-locked source (tests/_xfer.py)
        t[offset:offset + raw.size] = torch.from_numpy(raw.copy()).pin_memory().cuda()
    torch.cuda.synchronize()      # the library's streams do not order after torch's
    return t, t.data_ptr() + offset


def _host(t, offset, like):
    h = torch.empty(like.nbytes, dtype=torch.uint8).pin_memory()
    h.copy_(t[offset:offset + like.nbytes])
    torch.cuda.synchronize()
    return _raw(h.numpy(), like.dtype)


def _raw(a, dtype=None):
    """Writable array over a private byte copy of `a` (padding bytes kept:
    numpy's copy() of structured arrays does not preserve them)."""
    return np.frombuffer(bytearray(a.tobytes()), dtype=dtype if dtype is not None else a.dtype)


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _check_dev(L, op, dt, a, b, off_in=0, off_io=0):
    a, b = _raw(a), _raw(b)
    exp = _raw(b)
    rc_o = oracle.reduce_local(h(op), h(dt), a, exp)
    assert rc_o == 0
    ta, pa = _dev(a, off_in)
    tb, pb = _dev(b, off_io)
    rc = L.msx_reduce_local_dev(pa, pb, a.size, h(dt), h(op), _stream())
    assert rc == 0, msx.last_error()
    torch.cuda.synchronize()
    got = _host(tb, off_io, b)
    ok = np.array_equal(np.frombuffer(got.tobytes(), np.uint8), np.frombuffer(exp.tobytes(), np.uint8))
    if not ok:
        bad = np.nonzero(np.frombuffer(got.tobytes(), np.uint8) != np.frombuffer(exp.tobytes(), np.uint8))[0]
        i = bad[0] // got.dtype.itemsize
        pytest.fail(f"{op} {dt} n={a.size} off=({off_in},{off_io}): elem {i}: "
                    f"in={a[i]!r} inout={b[i]!r} got={got[i]!r} exp={exp[i]!r} ({len(bad)} bad bytes)")


_PAIRS = None


def _pairs():
    global _PAIRS
    if _PAIRS is None:
        _PAIRS = legal_pairs(oracle)
    return _PAIRS


@pytest.mark.parametrize("pair", _pairs(), ids=lambda p: f"{p[0]}-{p[1]}")
def test_every_legal_pair_bit_exact(L, pair):
    op, dt = pair
    kind = KIND[dt]
    rng = np.random.default_rng(zlib.crc32(f"{op}/{dt}".encode()))
    for n in (1, 3, 17, 1000, 65537):
        a, b = gen(kind, op, n, rng), gen(kind, op, n, rng)
        _check_dev(L, op, dt, a, b)


@pytest.mark.parametrize("dt", ["MPI_FLOAT", "MPI_INT8_T", "MPI_SHORT", "MPI_DOUBLE", "MPI_DOUBLE_INT",
                                "MPI_C_DOUBLE_COMPLEX", "MPI_SHORT_INT"])
def test_unaligned_and_misaligned_pointers(L, dt):
    kind = KIND[dt]
    esz = itemsize(kind)
    op = "MPI_MAXLOC" if kind in msx.LOC_DTYPES else "MPI_SUM"
    rng = np.random.default_rng(7)
    for n in (5, 4099):
        a, b = gen(kind, op, n, rng), gen(kind, op, n, rng)
        for off_in, off_io in ((esz, esz), (0, esz), (esz * 3, 0), (8, 8)):
            if off_in % min(esz, 8) or off_io % min(esz, 8):
                continue
            _check_dev(L, op, dt, a, b, off_in, off_io)


def test_realigned_operands_every_pair(L):
    # k_combine_shift: `in` and `inout` element-aligned at different offsets from
    # 16-byte alignment (every relative shift a type allows), every legal pair,
    # sizes around the 3-vector threshold and a ragged larger one
    rng = np.random.default_rng(71)
    for op, dt in legal_pairs(oracle):
        kind = KIND[dt]
        esz = itemsize(kind)
        if esz >= 16:
            continue
        for n in (3 * (16 // esz) - 1, 3 * (16 // esz) + 1, 5003):
            a, b = gen(kind, op, n, rng), gen(kind, op, n, rng)
            for off_in, off_io in ((esz, 0), (0, esz), (16 - esz, 2 * esz % 16)):
                if off_in % 16 == off_io % 16:
                    continue
                _check_dev(L, op, dt, a, b, off_in, off_io)
    # byte data at every byte shift (bitwise ops run on raw bytes)
    for shift in range(1, 16):
        a = rng.integers(0, 256, 4099, dtype=np.uint8)
        b = rng.integers(0, 256, 4099, dtype=np.uint8)
        _check_dev(L, "MPI_BXOR", "MPI_BYTE", a, b, shift, 0)
        _check_dev(L, "MPI_SUM", "MPI_INT8_T", a.view(np.int8), b.view(np.int8), 0, shift)


def test_realigned_operands_full_size(L):
    # 256 MiB fp32 SUM with `in` 4 bytes off: bit-exact vs torch (one IEEE add)
    n = (64 << 20) - 4
    g = torch.Generator(device="cuda").manual_seed(11)
    a = torch.rand(n + 4, device="cuda", generator=g)
    b = torch.rand(n, device="cuda", generator=g)
    exp = b + a[1:n + 1]
    torch.cuda.synchronize()
    assert L.msx_reduce_local_dev(a.data_ptr() + 4, b.data_ptr(), n, C.MPI_FLOAT, C.MPI_SUM, _stream()) == 0
    torch.cuda.synchronize()
    assert torch.equal(b.view(torch.int32), exp.view(torch.int32))


def test_loc_whole_struct_copy_includes_padding(L):
    # loctype `*this = rhs` (op.cpp:327) copies the whole struct
    rng = np.random.default_rng(9)
    for dt, kind in (("MPI_DOUBLE_INT", "di"), ("MPI_SHORT_INT", "si")):
        n = 4096
        a, b = gen(kind, "MPI_MAXLOC", n, rng), gen(kind, "MPI_MAXLOC", n, rng)
        ab = np.frombuffer(a.tobytes(), np.uint8).copy()
        bb = np.frombuffer(b.tobytes(), np.uint8).copy()
        isz = a.dtype.itemsize
        pad = [i for i in range(isz) if i not in set(range(0, a.dtype["v"].itemsize)) | set(
            range(a.dtype.fields["l"][1], a.dtype.fields["l"][1] + 4))]
        for pbyte in pad:
            ab[pbyte::isz] = rng.integers(0, 256, n, dtype=np.uint8)
            bb[pbyte::isz] = rng.integers(0, 256, n, dtype=np.uint8)
        a2 = _raw(ab, a.dtype)
        b2 = _raw(bb, a.dtype)
        _check_dev(L, "MPI_MAXLOC", dt, a2, b2)
        _check_dev(L, "MPI_MINLOC", dt, a2, b2)


def test_known_answer_vectors_on_gpu(L):
    with open(os.path.join(os.path.dirname(__file__), "golden", "survey_kat.json")) as f:
        kat = json.load(f)
    case = next(c for c in kat["cases"] if c["id"] == "int_sum_wrap_1MiB")
    i = np.arange(case["n"], dtype=np.int64)
    a = (7 * i - 3).astype(np.int32)
    b = (0x7FFFFFFF - i).astype(np.int32)
    ta, pa = _dev(a)
    tb, pb = _dev(b)
    assert L.msx_reduce_local_dev(pa, pb, a.size, C.MPI_INT, C.MPI_SUM, _stream()) == 0
    torch.cuda.synchronize()
    got = _host(tb, 0, b)
    assert got[0] == case["expect_first"] and got[-1] == case["expect_last"]
    case = next(c for c in kat["cases"] if c["id"] == "f32_max_nan_zero")
    to_f = lambda hx: np.array([int(x, 16) for x in hx], np.uint32).view(np.float32)
    a, b = to_f(case["in_f32_hex"]), to_f(case["inout_f32_hex"])
    ta, pa = _dev(a)
    tb, pb = _dev(b)
    assert L.msx_reduce_local_dev(pa, pb, 4, C.MPI_FLOAT, C.MPI_MAX, _stream()) == 0
    torch.cuda.synchronize()
    assert np.array_equal(_host(tb, 0, b).view(np.uint32), to_f(case["expect_f32_hex"]).view(np.uint32))


@pytest.mark.parametrize("pinned,mode", [(False, 0), (True, 0), (True, 1), (False, 1), (False, 2), (True, 2)])
def test_mpi_reduce_local_host_buffers_staged(L, pinned, mode):
    # the MPI path starts and ends in host memory: staged through HBM in chunks
    # (mode 1; pageable memory in mode 2), or combined in place over PCIe
    # (pinned memory in modes 0 and 2; pageable memory pinned for the call in
    # mode 0)
    assert L.msx_set_staging_chunk(1 << 20) == 0      # force many chunks
    assert L.msx_set_host_mode(mode) == 0
    rng = np.random.default_rng(11)
    for dt, op in (("MPI_FLOAT", "MPI_SUM"), ("MPI_UINT64_T", "MPI_BAND"), ("MPI_2INT", "MPI_MINLOC")):
        kind = KIND[dt]
        n = (3 << 20) // itemsize(kind) + 13
        a, b = gen(kind, op, n, rng), gen(kind, op, n, rng)
        exp = b.copy()
        oracle.reduce_local(h(op), h(dt), a, exp)
        if pinned:
            ta = torch.from_numpy(np.frombuffer(a.tobytes(), np.uint8).copy()).pin_memory()
            tb = torch.from_numpy(np.frombuffer(b.tobytes(), np.uint8).copy()).pin_memory()
            rc = L.MPI_Reduce_local(ta.data_ptr(), tb.data_ptr(), n, h(dt), h(op))
            got = np.frombuffer(tb.numpy().tobytes(), a.dtype)
        else:
            bb = b.copy()
            rc = L.MPI_Reduce_local(a.ctypes.data, bb.ctypes.data, n, h(dt), h(op))
            got = bb
        assert rc == 0, msx.last_error()
        assert got.tobytes() == exp.tobytes()
    assert L.msx_set_staging_chunk(64 << 20) == 0
    assert L.msx_set_host_mode(0) == 0


def test_pageable_operands_through_the_page_locked_ring(L):
    """Host mode 1 stages pageable operands through HBM; since round 5 their
    copies go through the library's page-locked ring (xfer_sync, 8 MiB slots,
    DESIGN.md §2), never HIP's pageable-copy path.  Operands of several ring
    slots with a ragged tail, at odd byte offsets, one staging chunk."""
    assert L.msx_set_staging_chunk(64 << 20) == 0
    assert L.msx_set_host_mode(1) == 0
    try:
        rng = np.random.default_rng(12)
        for dt, op, off in (("MPI_FLOAT", "MPI_SUM", 0), ("MPI_INT8_T", "MPI_BXOR", 3), ("MPI_DOUBLE", "MPI_MAX", 8)):
            kind = KIND[dt]
            n = (20 << 20) // itemsize(kind) + 7
            a, b = gen(kind, op, n + off, rng)[off:], gen(kind, op, n + off, rng)[off:]
            exp, b0 = b.copy(), b.tobytes()
            oracle.reduce_local(h(op), h(dt), a, exp)
            bb = b.copy() if off == 0 else b
            rc = L.MPI_Reduce_local(a.ctypes.data, bb.ctypes.data, n, h(dt), h(op))
            assert rc == 0, msx.last_error()
            assert bb.tobytes() == exp.tobytes(), (dt, op, off)
            # pageable `in`, page-locked `inout`: one operand through the ring, one by DMA
            tb = torch.from_numpy(np.frombuffer(b0, np.uint8).copy()).pin_memory()
            rc = L.MPI_Reduce_local(a.ctypes.data, tb.data_ptr(), n, h(dt), h(op))
            assert rc == 0, msx.last_error()
            assert tb.numpy().tobytes() == exp.tobytes(), (dt, op, off, "mixed")
    finally:
        assert L.msx_set_host_mode(0) == 0


def test_mpi_reduce_local_call_pin_edges(L):
    # host mode 0 pins pageable operands for the call: operands that share
    # pages (one pin of the union), unaligned starts and ragged ends, one
    # operand on the device, sizes either side of the 1 MiB pinning threshold, repeated
    # calls on the same buffers (the pin is released every time), and a
    # read-only `in` mapping the driver refuses to pin (staged instead)
    import mmap
    assert L.msx_set_host_mode(0) == 0
    rng = np.random.default_rng(21)
    big = rng.uniform(-1, 1, (5 << 20) // 4 + 77).astype(np.float32)
    for k in range(3):                                   # shared pages, odd offsets
        lo, n = 3 + k, (2 << 20) // 4 + 1001 * k + 5
        a = big[lo:lo + n]
        b = big[lo + n:lo + 2 * n].copy() if k == 2 else big[lo + n:lo + 2 * n]
        exp = b.copy()
        oracle.reduce_local(C.MPI_SUM, C.MPI_FLOAT, a.copy(), exp)
        assert L.MPI_Reduce_local(a.ctypes.data, b.ctypes.data, n, C.MPI_FLOAT, C.MPI_SUM) == 0, msx.last_error()
        assert b.tobytes() == exp.tobytes()
    for n in (1000, (1 << 20) // 8 - 1, (1 << 20) // 8, (3 << 20) // 8 + 3):   # around the 1 MiB threshold
        a = rng.integers(0, 2**63, n, dtype=np.uint64)
        b = rng.integers(0, 2**63, n, dtype=np.uint64)
        exp = b.copy()
        oracle.reduce_local(C.MPI_BXOR, C.MPI_UINT64_T, a, exp)
        for rep in range(2):                             # twice: pins released in between
            if rep:
                oracle.reduce_local(C.MPI_BXOR, C.MPI_UINT64_T, a, exp)
            assert L.MPI_Reduce_local(a.ctypes.data, b.ctypes.data, n, C.MPI_UINT64_T, C.MPI_BXOR) == 0
            assert np.array_equal(b, exp)
    n = (4 << 20) // 4                                   # device `in`, pageable `inout`
    a = rng.uniform(-1, 1, n).astype(np.float32)
    b = rng.uniform(-1, 1, n).astype(np.float32)
    exp = b.copy()
    oracle.reduce_local(C.MPI_MAX, C.MPI_FLOAT, a, exp)
    ta, pa = _dev(a)
    assert L.MPI_Reduce_local(pa, b.ctypes.data, n, C.MPI_FLOAT, C.MPI_MAX) == 0
    assert b.tobytes() == exp.tobytes()
    src = rng.integers(-2**31, 2**31, (8 << 20) // 4, dtype=np.int64).astype(np.int32)
    ro = mmap.mmap(-1, 8 << 20)                          # read-only `in`
    ro.write(src.tobytes())
    import ctypes as ct
    libc = ct.CDLL(None)
    addr = ct.addressof(ct.c_char.from_buffer(ro))
    assert libc.mprotect(ct.c_void_p(addr), ct.c_size_t(8 << 20), 1) == 0   # PROT_READ
    b = rng.integers(-2**31, 2**31, src.size, dtype=np.int64).astype(np.int32)
    exp = b.copy()
    oracle.reduce_local(C.MPI_SUM, C.MPI_INT, src, exp)
    assert L.MPI_Reduce_local(addr, b.ctypes.data, src.size, C.MPI_INT, C.MPI_SUM) == 0, msx.last_error()
    assert np.array_equal(b, exp)
    assert libc.mprotect(ct.c_void_p(addr), ct.c_size_t(8 << 20), 3) == 0


def test_mpi_reduce_local_device_and_mixed(L):
    rng = np.random.default_rng(12)
    n = 100003
    a = gen("f8", "MPI_PROD", n, rng)
    b = gen("f8", "MPI_PROD", n, rng)
    exp = b.copy()
    oracle.reduce_local(C.MPI_PROD, C.MPI_DOUBLE, a, exp)
    ta, pa = _dev(a)
    tb, pb = _dev(b)
    assert L.MPI_Reduce_local(pa, pb, n, C.MPI_DOUBLE, C.MPI_PROD) == 0
    assert _host(tb, 0, b).tobytes() == exp.tobytes()
    # host in, device inout
    tb, pb = _dev(b)
    assert L.MPI_Reduce_local(a.ctypes.data, pb, n, C.MPI_DOUBLE, C.MPI_PROD) == 0
    assert _host(tb, 0, b).tobytes() == exp.tobytes()
    # device in, host inout
    bb = b.copy()
    assert L.MPI_Reduce_local(pa, bb.ctypes.data, n, C.MPI_DOUBLE, C.MPI_PROD) == 0
    assert bb.tobytes() == exp.tobytes()


def test_user_op_on_device_buffers(L):
    UF = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int),
                          ctypes.POINTER(ctypes.c_int))

    def absmax(invec, inoutvec, n, dt):
        x = np.ctypeslib.as_array((ctypes.c_float * n[0]).from_address(invec))
        y = np.ctypeslib.as_array((ctypes.c_float * n[0]).from_address(inoutvec))
        y[:] = np.maximum(np.abs(x), np.abs(y))

    fn = UF(absmax)
    op = ctypes.c_int()
    assert L.MPI_Op_create(fn, 1, ctypes.byref(op)) == 0
    a = np.linspace(-5, 5, 1001).astype(np.float32)
    b = np.linspace(3, -3, 1001).astype(np.float32)
    ta, pa = _dev(a)
    tb, pb = _dev(b)
    assert L.MPI_Reduce_local(pa, pb, a.size, C.MPI_FLOAT, op.value) == 0
    assert np.array_equal(_host(tb, 0, b), np.maximum(np.abs(a), np.abs(b)))
    assert L.MPI_Op_free(ctypes.byref(op)) == 0


def test_tree_combine_reference_association(L):
    # msx_reduce_tree_dev: ((s0+s1)+(s2+s3))+((s4+s5)+(s6+s7)), left = inout
    rng = np.random.default_rng(13)
    n = 70001
    xs = [(rng.standard_normal(n) * 10.0 ** rng.integers(-7, 7, n)).astype(np.float32) for _ in range(8)]
    devs = [_dev(x) for x in xs]
    out = torch.zeros(n, dtype=torch.float32, device="cuda")
    for p in (2, 4, 8):
        arr = (ctypes.c_void_p * p)(*[d[1] for d in devs[:p]])
        assert L.msx_reduce_tree_dev(arr, p, out.data_ptr(), n, C.MPI_FLOAT, C.MPI_SUM, _stream()) == 0
        torch.cuda.synchronize()
        lv = list(xs[:p])
        while len(lv) > 1:
            lv = [lv[i] + lv[i + 1] for i in range(0, len(lv), 2)]
        assert np.array_equal(out.cpu().numpy().view(np.uint32), lv[0].view(np.uint32))
    # MAX with NaNs: the role of each operand matters (op.cpp:26)
    ys = [gen("f4", "MPI_MAX", n, rng) for _ in range(4)]
    dv = [_dev(y) for y in ys]
    arr = (ctypes.c_void_p * 4)(*[d[1] for d in dv])
    assert L.msx_reduce_tree_dev(arr, 4, out.data_ptr(), n, C.MPI_FLOAT, C.MPI_MAX, _stream()) == 0
    torch.cuda.synchronize()
    l0, l1 = ys[0].copy(), ys[2].copy()
    oracle.reduce_local(C.MPI_MAX, C.MPI_FLOAT, ys[1], l0)
    oracle.reduce_local(C.MPI_MAX, C.MPI_FLOAT, ys[3], l1)
    oracle.reduce_local(C.MPI_MAX, C.MPI_FLOAT, l1, l0)
    assert np.array_equal(out.cpu().numpy().view(np.uint32), l0.view(np.uint32))


@pytest.mark.parametrize("p", [2, 8, 16])
def test_tree_every_legal_pair(L, p):
    """msx_reduce_tree_dev for every legal (op, type) pair: p = 2 and 8 run the
    compile-time-source kernel, p = 16 the generic one; both must evaluate
    ((s0 op s1) op (s2 op s3)) ... with the left operand as `inout`, bit for
    bit as the oracle's pairwise Op<T> calls (edge values, ragged size)."""
    rng = np.random.default_rng(1000 + p)
    n = 1027
    for op, dt in legal_pairs(oracle):
        kind = KIND[dt]
        xs = [_raw(gen(kind, op, n, rng)) for _ in range(p)]
        dv = [_dev(x) for x in xs]
        arr = (ctypes.c_void_p * p)(*[d[1] for d in dv])
        out = torch.zeros(xs[0].nbytes + 64, dtype=torch.uint8, device="cuda")
        assert L.msx_reduce_tree_dev(arr, p, out.data_ptr(), n, h(dt), h(op), _stream()) == 0, msx.last_error()
        torch.cuda.synchronize()
        lv = [_raw(x) for x in xs]
        while len(lv) > 1:
            nxt = []
            for i in range(0, len(lv), 2):
                left = _raw(lv[i])
                assert oracle.reduce_local(h(op), h(dt), lv[i + 1], left) == 0
                nxt.append(left)
            lv = nxt
        got = out[:xs[0].nbytes].cpu().numpy().tobytes()
        assert got == lv[0].tobytes(), f"{op} {dt} p={p}"


def _oracle_tree(op, dt, srcs, P, pairmask, nleaves, chain):
    """The engine's tree evaluated with the oracle's combine (msx_tree_dev.h
    tree_eval): leaf k = srcs[2k] (op)= srcs[2k+1] when paired, then the
    balanced tree skipping absent leaves, left operand in the inout role; or
    the left-deep chain."""
    if chain:
        v = _raw(srcs[0])
        for k in range(1, P):
            assert oracle.reduce_local(h(op), h(dt), srcs[k], v) == 0
        return v
    nl = nleaves or P
    v = [None] * P
    for k in range(nl):
        v[k] = _raw(srcs[2 * k])
        if (pairmask >> k) & 1:
            assert oracle.reduce_local(h(op), h(dt), srcs[2 * k + 1], v[k]) == 0
    d = 1
    while d < P:
        for k in range(0, P - d, 2 * d):
            if k + d < nl:
                assert oracle.reduce_local(h(op), h(dt), v[k + d], v[k]) == 0
        d *= 2
    return v[0]


TREE_SPEC_PAIRS = [("MPI_SUM", "MPI_FLOAT"), ("MPI_SUM", "MPI_INT"), ("MPI_MAX", "MPI_DOUBLE"),
                   ("MPI_PROD", "MPI_C_FLOAT_COMPLEX"), ("MPI_MAXLOC", "MPI_2INT"), ("MPI_BXOR", "MPI_BYTE"),
                   ("MPI_LXOR", "MPI_C_BOOL"), ("MPI_MIN", "MPI_INT8_T")]


@pytest.mark.parametrize("pair", TREE_SPEC_PAIRS, ids=lambda p: f"{p[0]}-{p[1]}")
def test_tree_folds_absent_leaves_and_chains(L, pair):
    """The compile-time-leaf kernels of round 4 (tree_fixed MASKED: the
    non-power-of-two folds of p = 3, 5, 6, 7 and binomial trees with absent
    leaves; chains of 3-8 sources) against the oracle evaluating the same
    tree, bit for bit, every pattern the engine can produce for P = 2, 4, 8
    plus random ones, vector body + scalar tail."""
    op, dt = pair
    kind = KIND[dt]
    rng = np.random.default_rng(zlib.crc32(f"spec/{op}/{dt}".encode()))
    n = 4099
    srcs = [gen(kind, op, n, rng) for _ in range(16)]
    devs = [_dev(x) for x in srcs]
    ptrs = [p for _, p in devs]
    cases = []
    for P in (2, 4, 8):
        for nl in range(1, P + 1):
            cases.append((P, 0, nl, 0))                        # absent leaves (binomial trees)
        for pm in range(1, 1 << P) if P < 8 else rng.integers(1, 256, 24):
            cases.append((P, int(pm), P, 0))                   # folds (pairs)
        cases.append((P, int(rng.integers(0, 1 << P)), int(rng.integers(1, P + 1)), 0))
    for P in range(2, 9):
        cases.append((P, 0, 0, 1))                             # chains
    out = torch.zeros(n * srcs[0].itemsize + 64, dtype=torch.uint8, device="cuda")
    for P, pm, nl, chain in cases:
        ns = P if chain else 2 * P
        arr = (ctypes.c_void_p * ns)(*ptrs[:ns])
        rc = L.msx_reduce_tree_spec_dev(arr, P, pm, nl, chain, out.data_ptr(), n, h(dt), h(op), _stream())
        assert rc == 0, msx.last_error()
        torch.cuda.synchronize()
        got = _host(out, 0, srcs[0])
        exp = _oracle_tree(op, dt, srcs[:ns], P, pm, nl, chain)
        assert got.tobytes() == exp.tobytes(), (op, dt, P, hex(pm), nl, chain)


def test_tree_folds_dram_regime_fp32(L):
    """The masked kernel in its DRAM-regime form (source bytes above
    tree_nt_min: non-temporal loads, one-wave workgroups): p = 6's fold
    (P = 4, two pairs) and a p = 7 binomial tree (P = 8, 7 leaves) over 48 MiB
    sources, bit-exact against torch evaluating the same association."""
    n = 12 << 20
    g = torch.Generator(device="cuda").manual_seed(6)
    xs = [torch.rand(n, device="cuda", generator=g) * 2 - 1 for _ in range(8)]
    out = torch.empty_like(xs[0])
    torch.cuda.synchronize()
    # p = 6 allreduce fold: leaves 0, 1 paired
    arr = (ctypes.c_void_p * 8)(*[x.data_ptr() for x in xs])
    assert L.msx_reduce_tree_spec_dev(arr, 4, 0b11, 4, 0, out.data_ptr(), n, C.MPI_FLOAT, C.MPI_SUM,
                                      _stream()) == 0, msx.last_error()
    torch.cuda.synchronize()
    exp = ((xs[0] + xs[1]) + (xs[2] + xs[3])) + (xs[4] + (xs[6]))
    assert torch.equal(out.view(torch.int32), exp.view(torch.int32))
    # p = 7 binomial tree: leaves 0..6 of an 8-leaf tree (slots 2k)
    arr = (ctypes.c_void_p * 16)(*[xs[k // 2].data_ptr() if k % 2 == 0 else xs[0].data_ptr() for k in range(16)])
    assert L.msx_reduce_tree_spec_dev(arr, 8, 0, 7, 0, out.data_ptr(), n, C.MPI_FLOAT, C.MPI_SUM,
                                      _stream()) == 0, msx.last_error()
    torch.cuda.synchronize()
    exp = ((xs[0] + xs[1]) + (xs[2] + xs[3])) + ((xs[4] + xs[5]) + xs[6])
    assert torch.equal(out.view(torch.int32), exp.view(torch.int32))


@pytest.mark.parametrize("ngpus", [0, 1, 2, 8])
def test_reduce_local_multi_gpu_host_operands(L, ngpus):
    """msx_reduce_local_multi (one vector split over the node's
    GPUs, host operands over each GPU's PCIe link): bit-exact against the
    oracle for pageable and pinned host operands, a ragged count (range ends
    not on the 256-B grid), below and above the 1 MiB split threshold.  On a
    one-GPU box every ngpus clamps to that GPU; the driver's 8-GPU node runs
    the real split."""
    rng = np.random.default_rng(77 + ngpus)
    for n, op, dt in (((3 << 20) // 4 + 5, "MPI_SUM", "MPI_FLOAT"), (1000, "MPI_SUM", "MPI_FLOAT"),
                      ((5 << 20) // 8 + 3, "MPI_MAX", "MPI_DOUBLE"), ((2 << 20) + 7, "MPI_BXOR", "MPI_BYTE")):
        a, b = _raw(gen(KIND[dt], op, n, rng)), _raw(gen(KIND[dt], op, n, rng))
        exp = _raw(b)
        assert oracle.reduce_local(h(op), h(dt), a, exp) == 0
        for pinned in (False, True):
            if pinned:
                ta = torch.from_numpy(np.frombuffer(a.tobytes(), np.uint8).copy()).pin_memory()
                tb = torch.from_numpy(np.frombuffer(b.tobytes(), np.uint8).copy()).pin_memory()
                pa, pb = ta.data_ptr(), tb.data_ptr()
            else:
                ha, hb = _raw(a), _raw(b)
                pa, pb = ha.ctypes.data, hb.ctypes.data
            rc = L.msx_reduce_local_multi(pa, pb, n, h(dt), h(op), ngpus)
            assert rc == 0, msx.last_error()
            got = tb.numpy().tobytes() if pinned else hb.tobytes()
            assert got == exp.tobytes(), (op, dt, n, pinned, ngpus)
    # checks as MPI_Reduce_local: aliasing, unsupported pair
    x = np.ones(8, np.float32)
    assert L.msx_reduce_local_multi(x.ctypes.data, x.ctypes.data, 8, C.MPI_FLOAT, C.MPI_SUM, ngpus) == C.MPI_ERR_BUFFER
    assert L.msx_reduce_local_multi(x.ctypes.data, x.ctypes.data + 4, 1, C.MPI_BYTE, C.MPI_SUM, ngpus) == C.MPI_ERR_OP


@pytest.mark.parametrize("ngpus", [2, 3, 8])
def test_reduce_local_multi_split_on_one_device(L, ngpus):
    """The k-range split of msx_reduce_local_multi run on this box's one GPU
    (MSX_TEST_MULTI_SPLIT=1: range d on device d % visible): the call-scoped
    portable pins (listed like every call pin), the per-device aliases from the
    registered base plus the offset, 256-B range ends and the ragged tail --
    the code the 8-GPU node runs, minus the other devices.  Operands in
    separate buffers, and in one buffer (one pin covering both)."""
    os.environ["MSX_TEST_MULTI_SPLIT"] = "1"
    try:
        rng = np.random.default_rng(91 + ngpus)
        for n, op, dt in (((3 << 20) // 4 + 5, "MPI_SUM", "MPI_FLOAT"), ((5 << 20) // 8 + 3, "MPI_MAX", "MPI_DOUBLE"),
                          ((2 << 20) + 7, "MPI_BXOR", "MPI_BYTE")):
            a, b = _raw(gen(KIND[dt], op, n, rng)), _raw(gen(KIND[dt], op, n, rng))
            exp = _raw(b)
            assert oracle.reduce_local(h(op), h(dt), a, exp) == 0
            ha, hb = _raw(a), _raw(b)
            assert L.msx_reduce_local_multi(ha.ctypes.data, hb.ctypes.data, n, h(dt), h(op), ngpus) == 0, \
                msx.last_error()
            assert hb.tobytes() == exp.tobytes(), (op, dt, n, ngpus, "separate")
            both = np.concatenate([a, b])             # in and inout on shared pages: one pin
            assert L.msx_reduce_local_multi(both.ctypes.data, both.ctypes.data + a.nbytes, n, h(dt), h(op),
                                            ngpus) == 0, msx.last_error()
            assert both[n:].tobytes() == exp.tobytes(), (op, dt, n, ngpus, "shared pages")
            assert both[:n].tobytes() == a.tobytes()
    finally:
        del os.environ["MSX_TEST_MULTI_SPLIT"]
    # no pin outlives the call: the same pageable ranges pin again, alone
    x, y = _raw(gen(KIND["MPI_FLOAT"], "MPI_SUM", 1 << 20, rng)), _raw(gen(KIND["MPI_FLOAT"], "MPI_SUM", 1 << 20, rng))
    ye = _raw(y)
    assert oracle.reduce_local(C.MPI_SUM, C.MPI_FLOAT, x, ye) == 0
    assert L.MPI_Reduce_local(x.ctypes.data, y.ctypes.data, 1 << 20, C.MPI_FLOAT, C.MPI_SUM) == 0
    assert y.tobytes() == ye.tobytes()


def test_copy_geometries_exact(L):
    # the engine's local copy (msx_copy_dev): k_copy_segs' XCD-contiguous tiles
    # up to 16 MiB, k_copy_dram's one-wave dispatch order above; every byte
    # copied, nothing written past the end
    for nbytes in (4096, (1 << 20) + 48, (300 << 20) + 16):
        a = torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device="cuda")
        b = torch.zeros(nbytes + 64, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()      # the library's streams do not order after torch's
        assert L.msx_copy_dev(b.data_ptr(), a.data_ptr(), nbytes, _stream()) == 0, msx.last_error()
        torch.cuda.synchronize()
        assert torch.equal(b[:nbytes], a), nbytes
        assert int(b[nbytes:].count_nonzero()) == 0, nbytes
        del a, b


def test_probe_hbm_copy_modes_exact():
    # the bench-only probe library's copies (bench.py hbm_ceiling_probe): the
    # 16-B tile copy and the dispatch-order one-wave copy move every byte
    from msx import probe
    P = probe.lib()
    nbytes = (64 << 20) + 16
    a = torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device="cuda")
    for mode in (probe.COPY, probe.COPY_DISPATCH_ORDER):
        b = torch.zeros(nbytes, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        assert P.msxp_hbm(mode, a.data_ptr(), b.data_ptr(), nbytes, _stream()) == 0
        torch.cuda.synchronize()
        assert torch.equal(b, a), mode


def test_benchmark_size_fp32_sum_bit_exact(L):
    # config 2 (BASELINE.json): 256 MiB fp32 per operand, device resident.
    n = 64 << 20
    g = torch.Generator(device="cuda").manual_seed(0x5EED)
    a = torch.rand(n, device="cuda", generator=g) * 2 - 1
    b = torch.rand(n, device="cuda", generator=g) * 2 - 1
    exp = (a + b)       # one IEEE fp32 add per element (torch fp32 reference)
    assert L.msx_reduce_local_dev(a.data_ptr(), b.data_ptr(), n, C.MPI_FLOAT, C.MPI_SUM, _stream()) == 0
    torch.cuda.synchronize()
    assert torch.equal(b.view(torch.int32), exp.view(torch.int32))
    # and every measurement variant of the bench-only probe library (the same
    # combine body in other launch geometries, bench.py --sweep / cold launches)
    from msx import probe
    ref = b.clone()
    for name, v in probe.variants().items():
        c = b.clone()
        torch.cuda.synchronize()
        assert probe.lib().msxp_variant_run(v, a.data_ptr(), c.data_ptr(), n, _stream()) == 0, name
        torch.cuda.synchronize()
        assert torch.equal(c.view(torch.int32), (ref + a).view(torch.int32)), name


NAN_CASES_F32 = [0x7FC00001, 0xFFC00002, 0x7FA00003, 0xFF800000, 0x7F800000, 0x3F800000, 0x80000000, 0x00000001]


@pytest.mark.parametrize("dt", ["MPI_FLOAT", "MPI_DOUBLE", "MPI_C_FLOAT_COMPLEX", "MPI_C_DOUBLE_COMPLEX"])
@pytest.mark.parametrize("op", ["MPI_SUM", "MPI_PROD"])
def test_nan_payload_propagation_matches_reference_cpu(L, dt, op):
    """Two-NaN / inf-inf / signalling-NaN inputs: every NaN bit pattern must be
    the one the reference's x86 `inout op= in` produces (inout's NaN first,
    then in's, quieted; inf-inf = the x86 default NaN)."""
    if dt in ("MPI_FLOAT", "MPI_C_FLOAT_COMPLEX"):
        vals = np.array(NAN_CASES_F32, np.uint32).view(np.float32)
    else:
        vals = np.array([0x7FF8000000000001, 0xFFF8000000000002, 0x7FF4000000000003, 0xFFF0000000000000,
                         0x7FF0000000000000, 0x3FF0000000000000, 0x8000000000000000, 1], np.uint64).view(np.float64)
    a = np.repeat(vals, len(vals))
    b = np.tile(vals, len(vals))
    if "COMPLEX" in dt:
        ct = np.complex64 if vals.dtype == np.float32 else np.complex128
        ac = np.empty(a.size, ct); ac.real, ac.imag = a, b[::-1]
        bc = np.empty(b.size, ct); bc.real, bc.imag = b, a[::-1]
        a, b = ac, bc
    _check_dev(L, op, dt, a, b)


def test_plain_c_program_runs_on_the_gpu(tmp_path):
    """examples/reduce_local_demo.c (BASELINE configs[0] through the C ABI):
    gcc-built, linked with the library, bit-exact against the C loop."""
    import subprocess
    from test_abi import _build_c_demo
    exe = _build_c_demo(tmp_path)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120,
                       env={**os.environ, "MSX_SIZE": "1", "MSX_RANK": "0"})
    assert r.returncode == 0, r.stderr
    assert r.stdout.startswith("OK ")


def test_maximum_count_int_max_fp32(L):
    """Largest count the MPI API admits (count is an int, mpi.h:2352):
    MPI_Reduce_local over 2^31-1 fp32 (8 GiB per operand) on device buffers,
    checked in full against torch's fp32 add (one IEEE add per element) and
    at the ragged last elements.  The kernels index in 64 bits."""
    n = (1 << 31) - 1
    g = torch.Generator(device="cuda").manual_seed(7)
    a = torch.rand(n, device="cuda", generator=g)
    b = torch.rand(n, device="cuda", generator=g) - 0.5
    exp = a + b
    torch.cuda.synchronize()          # MPI calls take device buffers whose producers have finished
    assert L.MPI_Reduce_local(a.data_ptr(), b.data_ptr(), n, C.MPI_FLOAT, C.MPI_SUM) == 0
    torch.cuda.synchronize()
    assert torch.equal(b.view(torch.int32), exp.view(torch.int32))
    del a, b, exp
    torch.cuda.empty_cache()


def test_device_entry_beyond_4gib_bytes(L):
    """msx_reduce_local_dev takes a 64-bit count: 2^32 + 13 bytes of MPI_BXOR
    over MPI_BYTE (crosses every 32-bit byte-offset boundary), plus an odd
    start so the head/tail paths run too."""
    n = (1 << 32) + 13
    a = torch.empty(n + 1, dtype=torch.uint8, device="cuda").random_(0, 256)
    b = torch.empty(n + 1, dtype=torch.uint8, device="cuda").random_(0, 256)
    exp = b[1:] ^ a[1:]
    rc = L.msx_reduce_local_dev(a.data_ptr() + 1, b.data_ptr() + 1, n, C.MPI_BYTE, C.MPI_BXOR, _stream())
    assert rc == 0, msx.last_error()
    torch.cuda.synchronize()
    assert torch.equal(b[1:], exp)
    del a, b, exp
    torch.cuda.empty_cache()


_DRAM_CHILD = r'''
import ctypes, os, sys, zlib
sys.path.insert(0, os.path.join(REPO, "microsoft-mpi_amd")); sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import numpy as np, torch
import msx, oracle
from _cases import KIND, gen, h, legal_pairs
L = msx.init(errors_return=True)
s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
bad = []
for op, dt in legal_pairs(oracle):
    rng = np.random.default_rng(zlib.crc32(f"dram/{op}/{dt}".encode()))
    for n, off in ((17, 0), (65537, 0), (40000, 8)):
        a0, b0 = gen(KIND[dt], op, n, rng), gen(KIND[dt], op, n, rng)
        a = np.frombuffer(bytearray(a0.tobytes()), dtype=a0.dtype)
        b = np.frombuffer(bytearray(b0.tobytes()), dtype=b0.dtype)
        exp = np.frombuffer(bytearray(b.tobytes()), dtype=a.dtype)
        assert oracle.reduce_local(h(op), h(dt), a, exp) == 0
        if off % a.dtype.itemsize and off % 8:
            continue
        ta = torch.zeros(a.nbytes + off + 64, dtype=torch.uint8, device="cuda")
        tb = torch.zeros(b.nbytes + off + 64, dtype=torch.uint8, device="cuda")
        ta[off:off + a.nbytes] = torch.from_numpy(np.frombuffer(a.tobytes(), np.uint8).copy()).cuda()
        tb[off:off + b.nbytes] = torch.from_numpy(np.frombuffer(b.tobytes(), np.uint8).copy()).cuda()
        torch.cuda.synchronize()
        rc = L.msx_reduce_local_dev(ta.data_ptr() + off, tb.data_ptr() + off, n, h(dt), h(op), s)
        torch.cuda.synchronize()
        got = tb[off:off + b.nbytes].cpu().numpy().tobytes()
        if rc or got != exp.tobytes():
            bad.append(f"{op} {dt} n={n} off={off} rc={rc}")
print("DRAM_BAD", len(bad), bad[:5], flush=True)
'''


def test_dram_regime_kernel_every_pair(L, tmp_path):
    """k_combine_dram (operands above the Infinity Cache: one-wave workgroups
    in dispatch order) for every legal pair: MSX_TEST_COMBINE_DRAM_MIN=0 makes a
    child process route every vector-path call through it; bit-exact against
    the oracle, aligned and with an 8-byte common offset (head/tail paths).
    The in-process tests above cover it at its natural sizes (8 GiB fp32,
    4 GiB + 13 B BXOR)."""
    import subprocess
    import sys
    env = dict(os.environ, MSX_TEST_COMBINE_DRAM_MIN="0")
    r = subprocess.run([sys.executable, "-c", f"REPO={msx.REPO_ROOT!r}\n" + _DRAM_CHILD], capture_output=True,
                       text=True, timeout=300, env=env)
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("DRAM_BAD")]
    assert line and line[0].split()[1] == "0", (r.stdout + r.stderr)[-3000:]
