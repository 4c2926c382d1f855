"""Derived datatypes on the CPU: the oracle against the MPI-2.2 standard's worked
examples, the library's type attributes / envelopes against the oracle, and the
reference's argument-check order (api/mpi_datatype.cpp, api/mpi_pack.cpp).
No compute: MPI_Pack itself runs on the GPU (tests/test_gpu_dtype.py); here it
must fail loudly."""
import ctypes
import random

import numpy as np
import pytest

import msx
from oracle import msx_dtype_oracle as O

C = msx.C
c_int, c_i64 = ctypes.c_int, ctypes.c_int64


def ibuf(vals, ct=c_int):
    return (ct * max(len(vals), 1))(*vals)


# ---- a tiny recipe language shared by the oracle and the library ------------------
# ("basic", handle) | ("contig", n, r) | ("vector", n, blen, stride, r) |
# ("hvector", n, blen, bstride, r) | ("indexed", blens, disps, r) |
# ("hindexed", blens, bdisps, r) | ("iblock", blen, disps, r) |
# ("struct", blens, bdisps, [r...]) | ("resized", lb, extent, r) | ("dup", r) |
# ("subarray", sizes, subsizes, starts, order_c, r)
def build_oracle(r):
    k = r[0]
    if k == "basic":
        return O.marker(r[1]) if r[1] in (O.MPI_LB, O.MPI_UB) else O.predefined(r[1] & 0xFFFFFFFF)
    if k == "contig":
        return O.contiguous(r[1], build_oracle(r[2]))
    if k == "vector":
        return O.vector(r[1], r[2], r[3], build_oracle(r[4]))
    if k == "hvector":
        return O.hvector(r[1], r[2], r[3], build_oracle(r[4]))
    if k == "indexed":
        return O.indexed(r[1], r[2], build_oracle(r[3]))
    if k == "hindexed":
        return O.hindexed(r[1], r[2], build_oracle(r[3]))
    if k == "iblock":
        return O.indexed([r[1]] * len(r[2]), r[2], build_oracle(r[3]))
    if k == "struct":
        return O.struct(r[1], r[2], [build_oracle(x) for x in r[3]])
    if k == "resized":
        return O.resized(build_oracle(r[3]), r[1], r[2])
    if k == "dup":
        return build_oracle(r[1])
    if k == "subarray":
        return O.subarray(r[1], r[2], r[3], r[4], build_oracle(r[5]))
    if k == "darray":
        return O.darray(r[1], r[2], r[3], r[4], r[5], r[6], r[7], build_oracle(r[8]))
    raise ValueError(k)


def build_lib(L, r, keep):
    """Returns the handle; derived intermediates are appended to `keep`."""
    k = r[0]
    if k == "basic":
        return r[1]
    out = c_int()
    if k == "contig":
        rc = L.MPI_Type_contiguous(r[1], build_lib(L, r[2], keep), ctypes.byref(out))
    elif k == "vector":
        rc = L.MPI_Type_vector(r[1], r[2], r[3], build_lib(L, r[4], keep), ctypes.byref(out))
    elif k == "hvector":
        rc = L.MPI_Type_create_hvector(r[1], r[2], r[3], build_lib(L, r[4], keep), ctypes.byref(out))
    elif k == "indexed":
        rc = L.MPI_Type_indexed(len(r[1]), ibuf(r[1]), ibuf(r[2]), build_lib(L, r[3], keep), ctypes.byref(out))
    elif k == "hindexed":
        rc = L.MPI_Type_create_hindexed(len(r[1]), ibuf(r[1]), ibuf(r[2], c_i64), build_lib(L, r[3], keep),
                                        ctypes.byref(out))
    elif k == "iblock":
        rc = L.MPI_Type_create_indexed_block(len(r[2]), r[1], ibuf(r[2]), build_lib(L, r[3], keep),
                                             ctypes.byref(out))
    elif k == "struct":
        types = [build_lib(L, x, keep) for x in r[3]]
        rc = L.MPI_Type_create_struct(len(r[1]), ibuf(r[1]), ibuf(r[2], c_i64), ibuf(types), ctypes.byref(out))
    elif k == "resized":
        rc = L.MPI_Type_create_resized(build_lib(L, r[3], keep), r[1], r[2], ctypes.byref(out))
    elif k == "dup":
        rc = L.MPI_Type_dup(build_lib(L, r[1], keep), ctypes.byref(out))
    elif k == "subarray":
        n = len(r[1])
        rc = L.MPI_Type_create_subarray(n, ibuf(r[1]), ibuf(r[2]), ibuf(r[3]),
                                        C.MPI_ORDER_C if r[4] else C.MPI_ORDER_FORTRAN, build_lib(L, r[5], keep),
                                        ctypes.byref(out))
    elif k == "darray":
        n = len(r[3])
        rc = L.MPI_Type_create_darray(r[1], r[2], n, ibuf(r[3]), ibuf(r[4]), ibuf(r[5]), ibuf(r[6]),
                                      C.MPI_ORDER_C if r[7] else C.MPI_ORDER_FORTRAN, build_lib(L, r[8], keep),
                                      ctypes.byref(out))
    else:
        raise ValueError(k)
    assert rc == 0, (r, rc, msx.last_error())
    keep.append(out.value)
    return out.value


def lib_attrs(L, h):
    sz, lb, ext, tlb, text = c_i64(), c_i64(), c_i64(), c_i64(), c_i64()
    assert L.MPI_Type_size_x(h, ctypes.byref(sz)) == 0
    assert L.MPI_Type_get_extent(h, ctypes.byref(lb), ctypes.byref(ext)) == 0
    assert L.MPI_Type_get_true_extent(h, ctypes.byref(tlb), ctypes.byref(text)) == 0
    return sz.value, lb.value, ext.value, tlb.value, text.value


def oracle_attrs(t):
    return t.size, t.lb, t.extent, t.true_lb, t.true_ub - t.true_lb


def free_all(L, keep):
    for h in reversed(keep):
        x = c_int(h)
        assert L.MPI_Type_free(ctypes.byref(x)) == 0


BASICS = [C.MPI_INT, C.MPI_DOUBLE, C.MPI_CHAR, C.MPI_SHORT, C.MPI_FLOAT, C.MPI_LONG_LONG, C.MPI_BYTE]


def random_recipe(rng, depth=0):
    """Seeded random nesting of every constructor (small sizes)."""
    if depth >= 2 or rng.random() < 0.3:
        return ("basic", rng.choice(BASICS))
    k = rng.choice(["contig", "vector", "hvector", "indexed", "hindexed", "iblock", "struct", "resized",
                    "subarray", "dup", "darray"])
    sub = random_recipe(rng, depth + 1)
    if k == "contig":
        return ("contig", rng.randint(0, 4), sub)
    if k == "vector":
        return ("vector", rng.randint(1, 4), rng.randint(0, 3), rng.randint(-4, 6), sub)
    if k == "hvector":
        return ("hvector", rng.randint(1, 4), rng.randint(1, 3), rng.randint(-40, 64), sub)
    if k == "indexed":
        n = rng.randint(1, 4)
        return ("indexed", [rng.randint(0, 3) for _ in range(n)], [rng.randint(-3, 8) for _ in range(n)], sub)
    if k == "hindexed":
        n = rng.randint(1, 4)
        return ("hindexed", [rng.randint(0, 3) for _ in range(n)], [rng.randint(-16, 64) for _ in range(n)], sub)
    if k == "iblock":
        n = rng.randint(1, 4)
        return ("iblock", rng.randint(1, 3), [rng.randint(0, 8) for _ in range(n)], sub)
    if k == "struct":
        n = rng.randint(1, 3)
        subs = [random_recipe(rng, depth + 1) for _ in range(n)]
        return ("struct", [rng.randint(0, 3) for _ in range(n)], [rng.randint(0, 48) for _ in range(n)], subs)
    if k == "resized":
        return ("resized", rng.randint(-8, 8), rng.randint(1, 48), sub)
    if k == "subarray":
        nd = rng.randint(1, 3)
        sizes = [rng.randint(1, 5) for _ in range(nd)]
        subs = [rng.randint(0, s) for s in sizes]
        starts = [rng.randint(0, s - ss) for s, ss in zip(sizes, subs)]
        return ("subarray", sizes, subs, starts, rng.random() < 0.5, sub)
    if k == "darray":
        return random_darray(rng, sub)
    return ("dup", sub)


def random_darray(rng, sub):
    nd = rng.randint(1, 3)
    psizes = [rng.randint(1, 3) for _ in range(nd)]
    size = 1
    for q in psizes:
        size *= q
    gsizes = [rng.randint(1, 9) for _ in range(nd)]
    distribs, dargs = [], []
    for i in range(nd):
        d = rng.choice([C.MPI_DISTRIBUTE_BLOCK, C.MPI_DISTRIBUTE_CYCLIC, C.MPI_DISTRIBUTE_NONE])
        if d == C.MPI_DISTRIBUTE_NONE:
            psizes[i] = 1
        distribs.append(d)
        if d == C.MPI_DISTRIBUTE_BLOCK and rng.random() < 0.5:
            dargs.append(-(-gsizes[i] // psizes[i]) + rng.randint(0, 2))     # a block size that covers
        elif d == C.MPI_DISTRIBUTE_CYCLIC and rng.random() < 0.5:
            dargs.append(rng.randint(1, 3))
        else:
            dargs.append(C.MPI_DISTRIBUTE_DFLT_DARG)
    size = 1
    for q in psizes:
        size *= q
    return ("darray", size, rng.randrange(size), gsizes, distribs, dargs, psizes, rng.random() < 0.5, sub)


# ---------------------------------------------------------------------------------
def test_oracle_standard_examples():
    """MPI-2.2 §4.1 worked examples, restated through the oracle."""
    dbl, ch, flt = O.predefined(C.MPI_DOUBLE), O.predefined(C.MPI_CHAR), O.predefined(C.MPI_FLOAT)
    # oldtype {(double,0),(char,8)}, extent 16 (alignment padding of the struct)
    old = O.struct([1, 1], [0, 8], [dbl, ch])
    assert old.typemap == [(0, 8), (8, 1)] and old.extent == 16 and old.size == 9
    # Example 4.6: MPI_Type_vector(2, 3, 4, oldtype)
    v = O.vector(2, 3, 4, old)
    assert [d for d, _ in v.typemap] == [0, 8, 16, 24, 32, 40, 64, 72, 80, 88, 96, 104]
    assert (v.lb, v.extent) == (0, 112)
    # Example 4.7: MPI_Type_vector(3, 1, -2, oldtype)
    v = O.vector(3, 1, -2, old)
    assert [d for d, _ in v.typemap] == [0, 8, -32, -24, -64, -56]
    assert (v.lb, v.ub) == (-64, 16)
    # MPI_Type_contiguous(3, oldtype)
    c = O.contiguous(3, old)
    assert [d for d, _ in c.typemap] == [0, 8, 16, 24, 32, 40] and c.extent == 48
    # Example 4.9: MPI_Type_indexed(2, {3,1}, {4,0}, oldtype)
    ix = O.indexed([3, 1], [4, 0], old)
    assert [d for d, _ in ix.typemap] == [64, 72, 80, 88, 96, 104, 0, 8]
    assert (ix.lb, ix.ub) == (0, 112)
    # Example 4.11: struct {2 float at 0, 1 oldtype at 16, 3 char at 26}
    s = O.struct([2, 1, 3], [0, 16, 26], [flt, old, ch])
    assert s.typemap == [(0, 4), (4, 4), (16, 8), (24, 1), (26, 1), (27, 1), (28, 1)]
    assert (s.lb, s.extent, s.size) == (0, 32, 20)
    # resized: MPI_INT with lb -4, extent 16; true extent stays the data's
    r = O.resized(O.predefined(C.MPI_INT), -4, 16)
    assert (r.lb, r.extent, r.true_lb, r.true_ub) == (-4, 16, 0, 4)
    # subarray (C order) 4x5 doubles, 2x3 block at (1,2): rows at 56 and 96
    sa = O.subarray([4, 5], [2, 3], [1, 2], True, dbl)
    assert [d for d, _ in sa.typemap] == [56, 64, 72, 96, 104, 112]
    assert (sa.lb, sa.extent, sa.true_lb) == (0, 160, 56)


@pytest.mark.parametrize("seed", range(80))
def test_library_attributes_match_oracle(msxlib, seed):
    rng = random.Random(seed)
    r = random_recipe(rng)
    if r[0] == "basic":
        r = ("contig", 2, r)
    keep = []
    h = build_lib(msxlib, r, keep)
    t = build_oracle(r)
    assert lib_attrs(msxlib, h) == oracle_attrs(t), r
    free_all(msxlib, keep)


def test_library_standard_examples(msxlib):
    L = msxlib
    keep = []
    old = ("struct", [1, 1], [0, 8], [("basic", C.MPI_DOUBLE), ("basic", C.MPI_CHAR)])
    cases = [
        (("vector", 2, 3, 4, old), (54, 0, 112, 0, 105)),
        (("vector", 3, 1, -2, old), (27, -64, 80, -64, 73)),
        (("indexed", [3, 1], [4, 0], old), (36, 0, 112, 0, 105)),
        (("struct", [2, 1, 3], [0, 16, 26], [("basic", C.MPI_FLOAT), old, ("basic", C.MPI_CHAR)]),
         (20, 0, 32, 0, 29)),
        (("resized", -4, 16, ("basic", C.MPI_INT)), (4, -4, 16, 0, 4)),
        (("subarray", [4, 5], [2, 3], [1, 2], True, ("basic", C.MPI_DOUBLE)), (48, 0, 160, 56, 64)),
        (("subarray", [4, 5], [2, 3], [1, 2], False, ("basic", C.MPI_DOUBLE)), (48, 0, 160, 72, 80)),
        (("contig", 3, ("basic", C.MPI_DOUBLE_INT)), (36, 0, 48, 0, 44)),
    ]
    for r, want in cases:
        h = build_lib(L, r, keep)
        assert lib_attrs(L, h) == want, r
        assert oracle_attrs(build_oracle(r)) == want, r
    free_all(L, keep)


def test_darray_known_answers(msxlib):
    """Hand-derived darray layouts (MPI-2.2 §4.1.4 semantics; the reference's
    MPIR_Type_block / MPIR_Type_cyclic, mpid/datatype.cpp:409-637)."""
    L = msxlib
    I, B, Cy, N, D = C.MPI_INT, C.MPI_DISTRIBUTE_BLOCK, C.MPI_DISTRIBUTE_CYCLIC, C.MPI_DISTRIBUTE_NONE, \
        C.MPI_DISTRIBUTE_DFLT_DARG
    cases = [
        # 1-D block, 10 ints over 3 processes, rank 1: elements 4..7
        (("darray", 3, 1, [10], [B], [D], [3], True, ("basic", I)), [16, 20, 24, 28], (16, 0, 40, 16, 16)),
        # 1-D cyclic(2), rank 1: elements 2, 3, 8, 9
        (("darray", 3, 1, [10], [Cy], [2], [3], True, ("basic", I)), [8, 12, 32, 36], (16, 0, 40, 8, 32)),
        # 2-D C order, 4 x 6 block x cyclic over a 2 x 3 grid, rank 4: rows 2-3, columns 1 and 4
        (("darray", 6, 4, [4, 6], [B, Cy], [D, D], [2, 3], True, ("basic", I)), [52, 64, 76, 88],
         (16, 0, 96, 52, 40)),
        # the same grid in Fortran order: dimension 0 fastest
        (("darray", 6, 4, [4, 6], [B, Cy], [D, D], [2, 3], False, ("basic", I)), None, None),
        # MPI_DISTRIBUTE_NONE keeps the whole dimension
        (("darray", 2, 1, [3, 4], [N, B], [D, D], [1, 2], True, ("basic", I)), [8, 12, 24, 28, 40, 44],
         (24, 0, 48, 8, 40)),
    ]
    keep = []
    for r, disps, attrs in cases:
        t = build_oracle(r)
        h = build_lib(L, r, keep)
        if disps is not None:
            assert [d for d, _ in t.typemap] == disps, r
            assert oracle_attrs(t) == attrs, r
        assert lib_attrs(L, h) == oracle_attrs(t), r
    ni, na, nt, comb = c_int(), c_int(), c_int(), c_int()
    assert L.MPI_Type_get_envelope(h, ctypes.byref(ni), ctypes.byref(na), ctypes.byref(nt), ctypes.byref(comb)) == 0
    assert (ni.value, na.value, nt.value, comb.value) == (4 * 2 + 4, 0, 1, C.MPI_COMBINER_DARRAY)
    free_all(L, keep)
    # argument checks in the reference's order
    t = c_int()
    g, dd, ds, ps = ibuf([4]), ibuf([B]), ibuf([D]), ibuf([2])
    assert L.MPI_Type_create_darray(2, 0, 1, g, dd, ds, ps, C.MPI_ORDER_C, C.MPI_DATATYPE_NULL,
                                    ctypes.byref(t)) == C.MPI_ERR_TYPE
    assert L.MPI_Type_create_darray(2, -1, 1, g, dd, ds, ps, C.MPI_ORDER_C, I, ctypes.byref(t)) == C.MPI_ERR_ARG
    assert L.MPI_Type_create_darray(2, 0, 1, g, ibuf([99]), ds, ps, C.MPI_ORDER_C, I, ctypes.byref(t)) \
        == C.MPI_ERR_ARG
    assert L.MPI_Type_create_darray(2, 0, 1, g, dd, ibuf([0]), ps, C.MPI_ORDER_C, I, ctypes.byref(t)) \
        == C.MPI_ERR_ARG
    assert L.MPI_Type_create_darray(2, 0, 1, g, ibuf([N]), ds, ps, C.MPI_ORDER_C, I, ctypes.byref(t)) \
        == C.MPI_ERR_ARG                                                # NONE needs psize 1
    assert L.MPI_Type_create_darray(2, 0, 1, g, dd, ibuf([1]), ps, C.MPI_ORDER_C, I, ctypes.byref(t)) \
        == C.MPI_ERR_ARG                                                # 1 x 2 blocks < 4 elements
    assert L.MPI_Type_create_darray(2, 0, 1, g, dd, ds, ps, 7, I, ctypes.byref(t)) == C.MPI_ERR_ARG


def test_envelope_and_contents(msxlib):
    L = msxlib
    t = c_int()
    assert L.MPI_Type_vector(3, 2, 5, C.MPI_INT, ctypes.byref(t)) == 0
    ni, na, nt, comb = c_int(), c_int(), c_int(), c_int()
    assert L.MPI_Type_get_envelope(t, ctypes.byref(ni), ctypes.byref(na), ctypes.byref(nt), ctypes.byref(comb)) == 0
    assert (ni.value, na.value, nt.value, comb.value) == (3, 0, 1, C.MPI_COMBINER_VECTOR)
    ints, aints, types = (c_int * 3)(), (c_i64 * 1)(), (c_int * 1)()
    assert L.MPI_Type_get_contents(t, 3, 0, 1, ints, aints, types) == 0
    assert list(ints) == [3, 2, 5] and types[0] == C.MPI_INT
    # a predefined type is NAMED and has no contents (MpiaDatatypeValidateNotPermanent)
    assert L.MPI_Type_get_envelope(C.MPI_INT, ctypes.byref(ni), ctypes.byref(na), ctypes.byref(nt),
                                   ctypes.byref(comb)) == 0
    assert comb.value == C.MPI_COMBINER_NAMED
    assert L.MPI_Type_get_contents(C.MPI_INT, 0, 0, 0, None, None, None) == C.MPI_ERR_TYPE
    # struct contents carry the displacements and the member types
    s = c_int()
    assert L.MPI_Type_create_struct(2, ibuf([1, 2]), ibuf([0, 8], c_i64), ibuf([C.MPI_DOUBLE, t.value]),
                                    ctypes.byref(s)) == 0
    assert L.MPI_Type_get_envelope(s, ctypes.byref(ni), ctypes.byref(na), ctypes.byref(nt), ctypes.byref(comb)) == 0
    assert (ni.value, na.value, nt.value, comb.value) == (3, 2, 2, C.MPI_COMBINER_STRUCT)
    ints, aints, types = (c_int * 3)(), (c_i64 * 2)(), (c_int * 2)()
    assert L.MPI_Type_get_contents(s, 3, 2, 2, ints, aints, types) == 0
    assert list(ints) == [2, 1, 2] and list(aints) == [0, 8] and list(types) == [C.MPI_DOUBLE, t.value]
    # the vector is still alive while the struct (and the handed-out handle) refer to it
    assert L.MPI_Type_free(ctypes.byref(t)) == 0 and t.value == C.MPI_DATATYPE_NULL
    x = c_int(types[1])
    assert L.MPI_Type_free(ctypes.byref(x)) == 0          # the reference get_contents handed out
    assert L.MPI_Type_free(ctypes.byref(s)) == 0


def test_validation_order(msxlib):
    L = msxlib
    t = c_int()
    assert L.MPI_Type_contiguous(-1, C.MPI_INT, ctypes.byref(t)) == C.MPI_ERR_COUNT
    assert L.MPI_Type_contiguous(-1, C.MPI_INT, None) == C.MPI_ERR_COUNT        # count first
    assert L.MPI_Type_contiguous(1, C.MPI_INT, None) == C.MPI_ERR_ARG
    assert L.MPI_Type_contiguous(1, C.MPI_DATATYPE_NULL, ctypes.byref(t)) == C.MPI_ERR_TYPE
    assert L.MPI_Type_contiguous(1, 0x4C00FFFF, ctypes.byref(t)) == C.MPI_ERR_TYPE
    assert L.MPI_Type_vector(1, -1, 1, C.MPI_INT, ctypes.byref(t)) == C.MPI_ERR_ARG
    assert L.MPI_Type_vector(-1, -1, 1, C.MPI_INT, ctypes.byref(t)) == C.MPI_ERR_COUNT
    assert L.MPI_Type_indexed(1, None, ibuf([0]), C.MPI_INT, ctypes.byref(t)) == C.MPI_ERR_ARG
    assert L.MPI_Type_indexed(1, ibuf([-1]), ibuf([0]), C.MPI_DATATYPE_NULL, ctypes.byref(t)) == C.MPI_ERR_TYPE
    assert L.MPI_Type_indexed(1, ibuf([-1]), ibuf([0]), C.MPI_INT, ctypes.byref(t)) == C.MPI_ERR_ARG
    assert L.MPI_Type_create_struct(1, ibuf([1]), ibuf([0], c_i64), ibuf([C.MPI_DATATYPE_NULL]),
                                    ctypes.byref(t)) == C.MPI_ERR_TYPE
    sizes = ibuf([4, 4])
    assert L.MPI_Type_create_subarray(0, sizes, sizes, ibuf([0, 0]), C.MPI_ORDER_C, C.MPI_INT,
                                      ctypes.byref(t)) == C.MPI_ERR_ARG
    assert L.MPI_Type_create_subarray(2, sizes, ibuf([5, 1]), ibuf([0, 0]), C.MPI_ORDER_C, C.MPI_INT,
                                      ctypes.byref(t)) == C.MPI_ERR_ARG
    assert L.MPI_Type_create_subarray(2, sizes, ibuf([2, 2]), ibuf([3, 0]), C.MPI_ORDER_C, C.MPI_INT,
                                      ctypes.byref(t)) == C.MPI_ERR_ARG
    assert L.MPI_Type_create_subarray(2, sizes, ibuf([2, 2]), ibuf([0, 0]), 99, C.MPI_INT,
                                      ctypes.byref(t)) == C.MPI_ERR_ARG
    # predefined types are permanent: free fails, commit is a no-op
    x = c_int(C.MPI_INT)
    assert L.MPI_Type_free(ctypes.byref(x)) == C.MPI_ERR_TYPE
    x = c_int(C.MPI_FLOAT_INT)
    assert L.MPI_Type_free(ctypes.byref(x)) == C.MPI_ERR_TYPE
    x = c_int(C.MPI_INT)
    assert L.MPI_Type_commit(ctypes.byref(x)) == 0
    assert L.MPI_Type_commit(None) == C.MPI_ERR_ARG
    # a freed handle is no longer a datatype
    assert L.MPI_Type_contiguous(2, C.MPI_INT, ctypes.byref(t)) == 0
    stale = t.value
    assert L.MPI_Type_free(ctypes.byref(t)) == 0
    sz = c_int()
    assert L.MPI_Type_size(stale, ctypes.byref(sz)) == C.MPI_ERR_TYPE


def test_pack_checks_and_sizes(msxlib):
    L = msxlib
    t = c_int()
    assert L.MPI_Type_vector(4, 1, 2, C.MPI_DOUBLE, ctypes.byref(t)) == 0
    size = c_int()
    assert L.MPI_Pack_size(3, t, C.MPI_COMM_WORLD, ctypes.byref(size)) == C.MPI_ERR_TYPE   # uncommitted
    assert L.MPI_Type_commit(ctypes.byref(t)) == 0
    assert L.MPI_Pack_size(3, t, C.MPI_COMM_WORLD, ctypes.byref(size)) == 0 and size.value == 96
    assert L.MPI_Pack_size(1 << 28, C.MPI_DOUBLE, C.MPI_COMM_WORLD, ctypes.byref(size)) == 0
    assert size.value == C.MPI_UNDEFINED                                                   # > INT_MAX
    assert L.MPI_Pack_size(-1, t, C.MPI_COMM_WORLD, ctypes.byref(size)) == C.MPI_ERR_COUNT
    src = np.zeros(64, np.float64)
    out = np.zeros(96, np.uint8)
    pos = c_int(0)
    # output too small for 3 instances -> MPI_ERR_ARG before any data moves
    assert L.MPI_Pack(src.ctypes.data, 3, t, out.ctypes.data, 64, ctypes.byref(pos), C.MPI_COMM_WORLD) \
        == C.MPI_ERR_ARG
    assert L.MPI_Pack(src.ctypes.data, 1, t, out.ctypes.data, 96, None, C.MPI_COMM_WORLD) == C.MPI_ERR_ARG
    pos = c_int(-1)
    assert L.MPI_Pack(src.ctypes.data, 1, t, out.ctypes.data, 96, ctypes.byref(pos), C.MPI_COMM_WORLD) \
        == C.MPI_ERR_ARG
    pos = c_int(0)
    assert L.MPI_Pack(src.ctypes.data, 0, t, out.ctypes.data, 96, ctypes.byref(pos), C.MPI_COMM_WORLD) == 0
    assert pos.value == 0
    assert L.MPI_Unpack(out.ctypes.data, 0, ctypes.byref(pos), src.ctypes.data, 1, t, C.MPI_COMM_WORLD) == 0
    assert L.MPI_Unpack(out.ctypes.data, -1, ctypes.byref(pos), src.ctypes.data, 1, t, C.MPI_COMM_WORLD) \
        == C.MPI_ERR_COUNT
    assert L.MPI_Type_free(ctypes.byref(t)) == 0


def test_pack_without_gpu_fails_loudly(msxlib):
    """MPI_Pack moves bytes with the gfx950 kernel; with no GPU it must fail,
    not fall back to a CPU copy."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present: covered by tests/test_gpu_dtype.py")
    L = msxlib
    t = c_int()
    assert L.MPI_Type_vector(4, 1, 2, C.MPI_DOUBLE, ctypes.byref(t)) == 0
    assert L.MPI_Type_commit(ctypes.byref(t)) == 0
    src = np.arange(8, dtype=np.float64)
    out = np.zeros(32, np.uint8)
    pos = c_int(0)
    rc = L.MPI_Pack(src.ctypes.data, 1, t, out.ctypes.data, 32, ctypes.byref(pos), C.MPI_COMM_WORLD)
    assert rc == C.MPI_ERR_OTHER and pos.value == 0 and not out.any()
    assert L.MPI_Type_free(ctypes.byref(t)) == 0


def test_pair_type_size_is_data_bytes(msxlib):
    """MPI_Type_size counts data bytes (SetTypeCharacteristics,
    datatype.cpp:1282-1293): 12 for MPI_DOUBLE_INT, whose extent (element
    stride, msx_type_size) is 16; 6 / 8 for MPI_SHORT_INT."""
    L = msxlib
    for dt, size, ext in ((C.MPI_DOUBLE_INT, 12, 16), (C.MPI_SHORT_INT, 6, 8), (C.MPI_FLOAT_INT, 8, 8),
                          (C.MPI_2INT, 8, 8), (C.MPI_DOUBLE, 8, 8)):
        sz, lb, ex = c_int(), c_i64(), c_i64()
        assert L.MPI_Type_size(dt, ctypes.byref(sz)) == 0 and sz.value == size
        assert L.MPI_Type_get_extent(dt, ctypes.byref(lb), ctypes.byref(ex)) == 0
        assert (lb.value, ex.value) == (0, ext)
        assert L.msx_type_size(dt) == ext


def test_huge_strided_vector_stays_compact(msxlib):
    """A vector of 2^30 single-element blocks keeps its run list compact (first,
    length, stride): built instantly with the reference's attributes.  Using it
    inside another constructor expands the list, past the 2^25-run limit ->
    MPI_ERR_NO_MEM, a clean error rather than an allocation of 16 GiB."""
    import time
    L = msxlib
    t = c_int()
    t0 = time.perf_counter()
    assert L.MPI_Type_vector(1 << 30, 1, 2, C.MPI_FLOAT, ctypes.byref(t)) == 0
    assert time.perf_counter() - t0 < 0.5
    assert lib_attrs(L, t.value) == (4 << 30, 0, ((1 << 30) - 1) * 8 + 4, 0, ((1 << 30) - 1) * 8 + 4)
    assert L.MPI_Type_commit(ctypes.byref(t)) == 0
    s = c_int()
    assert L.MPI_Type_create_struct(2, ibuf([1, 1]), ibuf([0, 1 << 34], c_i64), ibuf([t.value, C.MPI_INT]),
                                    ctypes.byref(s)) == C.MPI_ERR_NO_MEM
    # a contiguous run of them merges into one run (no list at all)
    u = c_int()
    assert L.MPI_Type_vector(1 << 30, 4, 4, C.MPI_FLOAT, ctypes.byref(u)) == 0
    assert lib_attrs(L, u.value) == (16 << 30, 0, 16 << 30, 0, 16 << 30)
    assert L.MPI_Type_free(ctypes.byref(t)) == 0 and L.MPI_Type_free(ctypes.byref(u)) == 0


def test_vector_of_vector_and_3d_subarray_stay_compact(msxlib):
    """Two-level compact form: an hvector (one copy per block) of a strided
    vector keeps (first, length, stride, n, stride2, n2) instead of n * n2
    explicit runs -- 2^30 runs here, 32x the explicit limit, built and
    committed at once with the reference's attributes; likewise a 3-D
    subarray of a 2^40-byte array (its closing LB/UB struct keeps the form)."""
    import time
    L = msxlib
    inner, outer = c_int(), c_int()
    t0 = time.perf_counter()
    assert L.MPI_Type_vector(1 << 15, 1, 2, C.MPI_FLOAT, ctypes.byref(inner)) == 0
    assert L.MPI_Type_create_hvector(1 << 15, 1, 1 << 18, inner.value, ctypes.byref(outer)) == 0
    assert L.MPI_Type_commit(ctypes.byref(outer)) == 0
    ext_in = ((1 << 15) - 1) * 8 + 4
    ext = ((1 << 15) - 1) * (1 << 18) + ext_in
    assert lib_attrs(L, outer.value) == (4 << 30, 0, ext, 0, ext)
    sub = c_int()
    dims, subs, starts = [1 << 12, 1 << 13, 1 << 13], [1 << 11, 1 << 12, 1 << 12], [5, 7, 9]
    assert L.MPI_Type_create_subarray(3, ibuf(dims), ibuf(subs), ibuf(starts), C.MPI_ORDER_C, C.MPI_FLOAT,
                                      ctypes.byref(sub)) == 0
    assert L.MPI_Type_commit(ctypes.byref(sub)) == 0
    assert time.perf_counter() - t0 < 0.5
    first = ((5 * (1 << 13) + 7) * (1 << 13) + 9) * 4
    tl = first
    tu = first + (((1 << 11) - 1) * (1 << 13) + (1 << 12) - 1) * (1 << 13) * 4 + (1 << 12) * 4
    assert lib_attrs(L, sub.value) == ((1 << 35) * 4, 0, (1 << 38) * 4, tl, tu - tl)
    for h in (inner, outer, sub):
        assert L.MPI_Type_free(ctypes.byref(h)) == 0


UF = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int),
                      ctypes.POINTER(ctypes.c_int))


def make_typed_sub_op(L, t):
    """A user function that walks the datatype's type map (from the oracle)
    and computes inout = in - inout element by element, as a user of a derived
    datatype would write it; it checks it received the handle it expects."""
    seen = []

    def fn(invec, inoutvec, n, dt):
        seen.append((n[0], dt[0]))
        for i in range(n[0]):
            for d, sz in t["map"].typemap:
                off = i * t["map"].extent + d
                x = ctypes.c_int.from_address(invec + off)
                y = ctypes.c_int.from_address(inoutvec + off)
                y.value = x.value - y.value
    cb = UF(fn)
    op = c_int()
    assert L.MPI_Op_create(cb, 0, ctypes.byref(op)) == 0
    return op, cb, seen


def test_reduce_local_user_op_on_derived_type(msxlib):
    """MPI_Reduce_local with a user op and a committed derived datatype calls
    the user function once with (in, inout, count, handle) on the typed buffers
    (MPID_Uop_call, api/mpi_reduce.cpp:361); a builtin op rejects the derived
    type with MPI_ERR_OP (the check table), an uncommitted one MPI_ERR_TYPE."""
    L = msxlib
    r = ("indexed", [2, 1, 3], [0, 4, 7], ("basic", C.MPI_INT))
    keep = []
    h = build_lib(L, r, keep)
    t = {"map": build_oracle(r)}
    op, cb, seen = make_typed_sub_op(L, t)
    a = np.arange(40, dtype=np.int32)
    b = np.full(40, 100, dtype=np.int32)
    assert L.MPI_Reduce_local(a.ctypes.data, b.ctypes.data, 3, h, op.value) == C.MPI_ERR_TYPE   # uncommitted
    x = c_int(h)
    assert L.MPI_Type_commit(ctypes.byref(x)) == 0
    assert L.MPI_Reduce_local(a.ctypes.data, b.ctypes.data, 3, h, C.MPI_SUM) == C.MPI_ERR_OP
    assert L.MPI_Reduce_local(a.ctypes.data, b.ctypes.data, 3, h, op.value) == 0
    assert seen == [(3, h)]
    exp = np.full(40, 100, dtype=np.int32)
    idx = [i * t["map"].extent // 4 + d // 4 for i in range(3) for d, _ in t["map"].typemap]
    exp[idx] = a[idx] - 100
    assert b.tolist() == exp.tolist()
    assert L.MPI_Op_free(ctypes.byref(op)) == 0
    free_all(L, keep)
