"""GPU parity of the derived-datatype engine (msx_pack.hip) against the oracle.

MPI_Pack / MPI_Unpack move bytes with the gfx950 granule-map kernels; the
oracle (oracle/msx_dtype_oracle.py) gathers / scatters the MPI type map element
by element.  Byte movement is exact, so every check is bit-exact.  Covered:
every constructor nested at random (seeded), negative displacements and
strides, lb shifts, holes that unpack must preserve, host (pageable) and device
buffers, odd base addresses (1-byte granules), and size-independent properties
at large sizes (pack of a subarray == torch's slice; unpack(pack(x)) == x on
the type map).
"""
import ctypes
import random

import numpy as np
import pytest

import msx
from oracle import msx_dtype_oracle as O
from test_dtype_cpu import build_lib, build_oracle, free_all, random_recipe

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

C = msx.C
c_int = ctypes.c_int


@pytest.fixture(scope="module")
def L():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    lib = msx.init(errors_return=True)
    assert lib.msx_device_count() > 0
    return lib


def _commit(L, r, keep):
    h = build_lib(L, r, keep)
    x = c_int(h)
    assert L.MPI_Type_commit(ctypes.byref(x)) == 0
    return h


def _layout(t, count, misalign):
    lo, hi = O.span(t, count)
    base = -lo + misalign            # byte index of the buffer address inside the array
    return base, hi - lo + misalign + 16


def _overlaps(t, count):
    """A receive type map with overlapping entries is erroneous in MPI (the
    last write is unspecified); such types are checked on pack only."""
    seen = set()
    for i in range(count):
        for d, sz in t.typemap:
            for b in range(i * t.extent + d, i * t.extent + d + sz):
                if b in seen:
                    return True
                seen.add(b)
    return False


def _recipes(n, seed0):
    out = []
    seed = seed0
    while len(out) < n:
        rng = random.Random(seed)
        seed += 1
        r = random_recipe(rng)
        if r[0] == "basic":
            r = ("vector", 3, 2, 3, r)
        t = build_oracle(r)
        if t.size == 0:
            continue
        out.append((r, rng.randint(1, 5), rng.choice([0, 0, 1, 3, 8])))
    return out


@pytest.mark.parametrize("case", _recipes(40, 1000))
def test_pack_unpack_host_buffers(L, case):
    r, count, mis = case
    keep = []
    h = _commit(L, r, keep)
    t = build_oracle(r)
    base, nbytes = _layout(t, count, mis)
    rng = np.random.default_rng(len(keep) * 7919 + count)
    typed = rng.integers(0, 256, nbytes, dtype=np.uint8)
    want = O.pack(t, count, typed, base)
    out = np.zeros(want.size + 8, np.uint8)
    pos = c_int(3)                    # pack at a non-zero position
    rc = L.MPI_Pack(typed.ctypes.data + base, count, h, out.ctypes.data, out.size, ctypes.byref(pos),
                    C.MPI_COMM_WORLD)
    assert rc == 0, msx.last_error()
    assert pos.value == 3 + want.size
    assert np.array_equal(out[3:3 + want.size], want), r
    if _overlaps(t, count):
        free_all(L, keep)
        return
    # unpack random bytes into a buffer whose holes must survive
    src = rng.integers(0, 256, want.size + 3, dtype=np.uint8)
    dst = rng.integers(0, 256, nbytes, dtype=np.uint8)
    exp = dst.copy()
    O.unpack(t, count, src[3:], exp, base)
    pos = c_int(3)
    rc = L.MPI_Unpack(src.ctypes.data, src.size, ctypes.byref(pos), dst.ctypes.data + base, count, h,
                      C.MPI_COMM_WORLD)
    assert rc == 0, msx.last_error()
    assert pos.value == src.size
    assert np.array_equal(dst, exp), r
    free_all(L, keep)


@pytest.mark.parametrize("mode", [0, 2])      # 2: the one-wave tile form forced (msx_tune_pack)
@pytest.mark.parametrize("case", _recipes(25, 5000))
def test_pack_unpack_device_buffers(L, case, mode):
    assert L.msx_tune_pack(mode) == 0
    try:
        _pack_unpack_device(L, case)
    finally:
        assert L.msx_tune_pack(0) == 0


def _pack_unpack_device(L, case):
    r, count, mis = case
    keep = []
    h = _commit(L, r, keep)
    t = build_oracle(r)
    base, nbytes = _layout(t, count, mis)
    g = torch.Generator(device="cuda").manual_seed(count * 31 + mis)
    typed = torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device="cuda", generator=g)
    want = O.pack(t, count, typed.cpu().numpy(), base)
    out = torch.zeros(want.size, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    pos = c_int(0)
    rc = L.MPI_Pack(typed.data_ptr() + base, count, h, out.data_ptr(), out.numel(), ctypes.byref(pos),
                    C.MPI_COMM_WORLD)
    assert rc == 0, msx.last_error()
    assert np.array_equal(out.cpu().numpy(), want), r
    if _overlaps(t, count):
        free_all(L, keep)
        return
    dst = torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device="cuda", generator=g)
    exp = dst.cpu().numpy().copy()
    src = torch.randint(0, 256, (want.size,), dtype=torch.uint8, device="cuda", generator=g)
    O.unpack(t, count, src.cpu().numpy(), exp, base)
    pos = c_int(0)
    rc = L.MPI_Unpack(src.data_ptr(), src.numel(), ctypes.byref(pos), dst.data_ptr() + base, count, h,
                      C.MPI_COMM_WORLD)
    assert rc == 0, msx.last_error()
    assert np.array_equal(dst.cpu().numpy(), exp), r
    free_all(L, keep)


def test_pair_and_resized_types(L):
    """Pair types keep their padding out of the packed stream; a resized type
    with a negative lb packs from before the buffer address."""
    keep = []
    for r, count in [(("contig", 5, ("basic", C.MPI_DOUBLE_INT)), 7),
                     (("contig", 3, ("basic", C.MPI_SHORT_INT)), 4),
                     (("resized", -8, 24, ("basic", C.MPI_DOUBLE)), 9),
                     (("hvector", 4, 1, -24, ("basic", C.MPI_FLOAT_INT)), 3)]:
        h = _commit(L, r, keep)
        t = build_oracle(r)
        base, nbytes = _layout(t, count, 0)
        typed = np.random.default_rng(count).integers(0, 256, nbytes, dtype=np.uint8)
        want = O.pack(t, count, typed, base)
        out = np.zeros(want.size, np.uint8)
        pos = c_int(0)
        assert L.MPI_Pack(typed.ctypes.data + base, count, h, out.ctypes.data, out.size, ctypes.byref(pos),
                          C.MPI_COMM_WORLD) == 0, msx.last_error()
        assert np.array_equal(out, want), r
    free_all(L, keep)


def test_large_subarray_equals_torch_slice(L):
    """Size-independent property at 1 GiB: a 3-D C-order subarray of fp32
    packs to exactly torch's contiguous copy of the same slice, and unpacking
    it into a zeroed array restores the slice and nothing else."""
    n0, n1, n2 = 256, 1024, 1024                       # 1 GiB fp32
    s0, s1, s2 = 100, 700, 513                         # ragged inner rows (2052 B)
    st = (77, 300, 255)
    x = torch.randn(n0, n1, n2, device="cuda")
    keep = []
    h = _commit(L, ("subarray", [n0, n1, n2], [s0, s1, s2], list(st), True, ("basic", C.MPI_FLOAT)), keep)
    want = x[st[0]:st[0] + s0, st[1]:st[1] + s1, st[2]:st[2] + s2].contiguous()
    out = torch.empty_like(want)
    torch.cuda.synchronize()          # blocking MPI calls take buffers whose producers have finished
    pos = c_int(0)
    nb = want.numel() * 4
    assert L.MPI_Pack(x.data_ptr(), 1, h, out.data_ptr(), nb, ctypes.byref(pos), C.MPI_COMM_WORLD) == 0
    torch.cuda.synchronize()
    assert pos.value == nb
    assert torch.equal(out.view(torch.int32), want.view(torch.int32))
    y = torch.zeros_like(x)
    torch.cuda.synchronize()
    pos = c_int(0)
    assert L.MPI_Unpack(out.data_ptr(), nb, ctypes.byref(pos), y.data_ptr(), 1, h, C.MPI_COMM_WORLD) == 0
    torch.cuda.synchronize()
    mask = torch.zeros_like(x, dtype=torch.bool)
    mask[st[0]:st[0] + s0, st[1]:st[1] + s1, st[2]:st[2] + s2] = True
    assert torch.equal(y[mask], x[mask])
    assert not y[~mask].any()
    free_all(L, keep)


def test_large_vector_round_trip_general_layout(L):
    """An indexed type with irregular blocks (the binary-search path), 2^20
    instances on device buffers: unpack(pack(x)) touches exactly the type map."""
    keep = []
    r = ("indexed", [3, 1, 7, 2], [0, 5, 9, 20], ("basic", C.MPI_INT))
    h = _commit(L, r, keep)
    t = build_oracle(r)
    count = 1 << 20
    ext = t.extent
    x = torch.randint(-2**31, 2**31 - 1, (count * ext // 4,), dtype=torch.int32, device="cuda")
    packed = torch.empty(count * t.size // 4, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    pos = c_int(0)
    assert L.MPI_Pack(x.data_ptr(), count, h, packed.data_ptr(), packed.numel() * 4, ctypes.byref(pos),
                      C.MPI_COMM_WORLD) == 0
    idx = torch.tensor([d // 4 for d, _ in t.typemap], device="cuda")
    rows = (torch.arange(count, device="cuda") * (ext // 4)).unsqueeze(1) + idx.unsqueeze(0)
    assert torch.equal(packed, x[rows.reshape(-1)])
    y = torch.zeros_like(x)
    torch.cuda.synchronize()
    pos = c_int(0)
    assert L.MPI_Unpack(packed.data_ptr(), packed.numel() * 4, ctypes.byref(pos), y.data_ptr(), count, h,
                        C.MPI_COMM_WORLD) == 0
    torch.cuda.synchronize()
    assert torch.equal(y[rows.reshape(-1)], x[rows.reshape(-1)])
    y[rows.reshape(-1)] = 0
    assert not y.any()
    free_all(L, keep)


LONG_RUNS = [
    ("hindexed", [40, 3, 100], [0, 400, 1000], ("basic", C.MPI_INT)),
    ("subarray", [6, 7, 40], [3, 4, 33], [1, 2, 5], True, ("basic", C.MPI_DOUBLE)),
    ("subarray", [9, 50], [4, 31], [3, 7], False, ("basic", C.MPI_FLOAT)),
    ("struct", [64, 1, 20], [0, 512, 600], [("basic", C.MPI_DOUBLE), ("basic", C.MPI_CHAR),
                                            ("basic", C.MPI_SHORT)]),
]


@pytest.mark.parametrize("r", LONG_RUNS)
@pytest.mark.parametrize("mis", [0, 1, 4])
def test_long_run_layouts(L, r, mis):
    """Layouts with long runs take the wave-per-run kernel; checked against
    the oracle on host and device buffers, at several base alignments."""
    keep = []
    h = _commit(L, r, keep)
    t = build_oracle(r)
    for count in (1, 3):
        base, nbytes = _layout(t, count, mis)
        typed = np.random.default_rng(count + mis).integers(0, 256, nbytes, dtype=np.uint8)
        want = O.pack(t, count, typed, base)
        td = torch.from_numpy(typed).cuda()
        out = torch.zeros(want.size, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        pos = c_int(0)
        assert L.MPI_Pack(td.data_ptr() + base, count, h, out.data_ptr(), want.size, ctypes.byref(pos),
                          C.MPI_COMM_WORLD) == 0, msx.last_error()
        assert np.array_equal(out.cpu().numpy(), want), (r, count, mis)
        dst = np.random.default_rng(7).integers(0, 256, nbytes, dtype=np.uint8)
        exp = dst.copy()
        src = np.random.default_rng(8).integers(0, 256, want.size, dtype=np.uint8)
        O.unpack(t, count, src, exp, base)
        pos = c_int(0)
        assert L.MPI_Unpack(src.ctypes.data, src.size, ctypes.byref(pos), dst.ctypes.data + base, count, h,
                            C.MPI_COMM_WORLD) == 0, msx.last_error()
        assert np.array_equal(dst, exp), (r, count, mis)
    free_all(L, keep)


def test_compact_vector_beyond_explicit_run_limit(L):
    """2^27 strided blocks (4x the explicit run-list limit) pack straight from
    the compact (first, length, stride) form: MPI_Pack of every other fp32 of a
    1 GiB buffer equals torch's x[::2], and unpack restores exactly those."""
    n = 1 << 28
    x = torch.randn(n, device="cuda")
    t = c_int()
    assert L.MPI_Type_vector(n // 2, 1, 2, C.MPI_FLOAT, ctypes.byref(t)) == 0
    assert L.MPI_Type_commit(ctypes.byref(t)) == 0
    out = torch.empty(n // 2, device="cuda")
    torch.cuda.synchronize()
    pos = c_int(0)
    assert L.MPI_Pack(x.data_ptr(), 1, t.value, out.data_ptr(), 2 * n, ctypes.byref(pos), C.MPI_COMM_WORLD) == 0, \
        msx.last_error()
    torch.cuda.synchronize()
    bad = (out != x[::2]).nonzero().flatten()
    assert bad.numel() == 0, (bad.numel(), bad[:8].tolist(), bad[-4:].tolist())
    y = torch.zeros_like(x)
    torch.cuda.synchronize()
    pos = c_int(0)
    assert L.MPI_Unpack(out.data_ptr(), 2 * n, ctypes.byref(pos), y.data_ptr(), 1, t.value, C.MPI_COMM_WORLD) == 0
    torch.cuda.synchronize()
    assert torch.equal(y[::2], x[::2]) and not y[1::2].any()
    assert L.MPI_Type_free(ctypes.byref(t)) == 0


def test_two_level_compact_beyond_explicit_run_limit(L):
    """Two-level compact form: an hvector of 2^14 rows, each a vector of 2^13
    every-other fp32 -- 2^27 runs, 4x the explicit run-list limit -- packs
    from (first, len, stride, n, stride2, n2) alone: MPI_Pack of a 1 GiB buffer
    equals torch's x.view(2^14, 2^14)[:, ::2], unpack restores exactly it."""
    n = 1 << 28
    x = torch.randn(n, device="cuda")
    inner, t = c_int(), c_int()
    assert L.MPI_Type_vector(1 << 13, 1, 2, C.MPI_FLOAT, ctypes.byref(inner)) == 0
    assert L.MPI_Type_create_hvector(1 << 14, 1, (1 << 14) * 4, inner.value, ctypes.byref(t)) == 0
    assert L.MPI_Type_commit(ctypes.byref(t)) == 0
    want = x.view(1 << 14, 1 << 14)[:, ::2].reshape(-1)
    out = torch.empty(n // 2, device="cuda")
    torch.cuda.synchronize()
    pos = c_int(0)
    assert L.MPI_Pack(x.data_ptr(), 1, t.value, out.data_ptr(), 2 * n, ctypes.byref(pos), C.MPI_COMM_WORLD) == 0, \
        msx.last_error()
    torch.cuda.synchronize()
    assert pos.value == 2 * n
    bad = (out != want).nonzero().flatten()
    assert bad.numel() == 0, (bad.numel(), bad[:8].tolist())
    y = torch.zeros_like(x)
    torch.cuda.synchronize()
    pos = c_int(0)
    assert L.MPI_Unpack(out.data_ptr(), 2 * n, ctypes.byref(pos), y.data_ptr(), 1, t.value, C.MPI_COMM_WORLD) == 0
    torch.cuda.synchronize()
    assert torch.equal(y[::2], x[::2]) and not y[1::2].any()
    for h in (inner, t):
        assert L.MPI_Type_free(ctypes.byref(h)) == 0


@pytest.mark.parametrize("order", ["C", "F"])
def test_subarray_3d_two_level_form_matches_torch(L, order):
    """3-D subarrays (C and Fortran order) now keep the two-level compact form
    through their LB/UB struct: pack / unpack against torch slicing, with rows
    long enough for the run-parallel kernel and short enough for the granule
    map, device buffers."""
    for dims, sub, st in (((48, 64, 96), (20, 30, 40), (3, 5, 7)), ((40, 50, 6), (10, 20, 3), (1, 2, 3))):
        x = torch.randn(*dims, device="cuda")
        ia = lambda v: (ctypes.c_int * 3)(*v)
        t = c_int()
        o = C.MPI_ORDER_C if order == "C" else C.MPI_ORDER_FORTRAN
        d, s_, st_ = (dims, sub, st) if order == "C" else (dims[::-1], sub[::-1], st[::-1])
        assert L.MPI_Type_create_subarray(3, ia(d), ia(s_), ia(st_), o, C.MPI_FLOAT, ctypes.byref(t)) == 0
        assert L.MPI_Type_commit(ctypes.byref(t)) == 0
        want = x[st[0]:st[0] + sub[0], st[1]:st[1] + sub[1], st[2]:st[2] + sub[2]].reshape(-1)
        out = torch.empty(want.numel(), device="cuda")
        torch.cuda.synchronize()
        pos = c_int(0)
        assert L.MPI_Pack(x.data_ptr(), 1, t.value, out.data_ptr(), out.numel() * 4, ctypes.byref(pos),
                          C.MPI_COMM_WORLD) == 0, msx.last_error()
        torch.cuda.synchronize()
        assert torch.equal(out, want), (dims, order)
        y = torch.zeros_like(x)
        torch.cuda.synchronize()
        pos = c_int(0)
        assert L.MPI_Unpack(out.data_ptr(), out.numel() * 4, ctypes.byref(pos), y.data_ptr(), 1, t.value,
                            C.MPI_COMM_WORLD) == 0
        torch.cuda.synchronize()
        m = torch.zeros_like(x, dtype=torch.bool)
        m[st[0]:st[0] + sub[0], st[1]:st[1] + sub[1], st[2]:st[2] + sub[2]] = True
        assert torch.equal(y[m], x[m]) and not y[~m].any(), (dims, order)
        assert L.MPI_Type_free(ctypes.byref(t)) == 0


def test_reduce_local_user_op_derived_type_device_buffers(L):
    """User op + derived type on DEVICE buffers: the library stages the type's
    byte span through host memory around the user function; the bytes between
    mapped elements of inout come back unchanged."""
    from test_dtype_cpu import make_typed_sub_op
    r = ("hvector", 5, 2, 24, ("basic", C.MPI_INT))
    keep = []
    h = _commit(L, r, keep)
    t = {"map": build_oracle(r)}
    op, cb, seen = make_typed_sub_op(L, t)
    a = torch.arange(200, dtype=torch.int32, device="cuda")
    b = torch.full((200,), 7, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    assert L.MPI_Reduce_local(a.data_ptr() + 8, b.data_ptr() + 8, 4, h, op.value) == 0, msx.last_error()
    exp = np.full(200, 7, dtype=np.int32)
    idx = [2 + i * t["map"].extent // 4 + d // 4 for i in range(4) for d, _ in t["map"].typemap]
    exp[idx] = np.arange(200, dtype=np.int32)[idx] - 7
    assert b.cpu().numpy().tolist() == exp.tolist()
    assert seen == [(4, h)]
    assert L.MPI_Op_free(ctypes.byref(op)) == 0
    free_all(L, keep)


def test_type_freed_while_nonblocking_op_pending(L):
    """MPI_Type_free of a derived type used by a pending MPI_Iallreduce (user
    op, one-rank communicator: the non-contiguous local copy) only marks it:
    the request keeps a reference until it completes."""
    from test_dtype_cpu import make_typed_sub_op
    r = ("vector", 4, 2, 3, ("basic", C.MPI_INT))
    keep = []
    h = _commit(L, r, keep)
    t = {"map": build_oracle(r)}
    op, cb, seen = make_typed_sub_op(L, t)
    a = torch.arange(64, dtype=torch.int32, device="cuda")
    b = torch.full((64,), -1, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    req = c_int()
    assert L.MPI_Iallreduce(a.data_ptr(), b.data_ptr(), 2, h, op.value, C.MPI_COMM_WORLD, ctypes.byref(req)) == 0
    x = c_int(h)
    assert L.MPI_Type_free(ctypes.byref(x)) == 0            # user frees it while pending
    assert L.MPI_Wait(ctypes.byref(req), ctypes.c_void_p(1)) == 0, msx.last_error()
    idx = [i * t["map"].extent // 4 + d // 4 for i in range(2) for d, _ in t["map"].typemap]
    exp = np.full(64, -1, np.int32)
    exp[idx] = np.arange(64, dtype=np.int32)[idx]
    assert b.cpu().numpy().tolist() == exp.tolist()
    assert L.MPI_Op_free(ctypes.byref(op)) == 0
