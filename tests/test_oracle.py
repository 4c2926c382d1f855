"""CPU: pin the oracle (C restatement of op.cpp) against the reference's
known-answer outputs, and check its multi-rank schedule simulator against the
association orders the reference's schedules produce (SURVEY.md §8 notes)."""
import json
import os

import numpy as np
import pytest

import msx
import oracle
from _cases import KIND, NON_REDUCIBLE, OPS, gen, h, np_dtype

C = msx.C
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _f32(hexes):
    return np.array([int(x, 16) for x in hexes], dtype=np.uint32).view(np.float32)


def _kat():
    with open(os.path.join(GOLD, "survey_kat.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("case", _kat()["cases"], ids=lambda c: c["id"])
def test_oracle_known_answers(case):
    op, dt = h(case["op"]), h(case["dt"])
    kind = KIND[case["dt"]]
    if "in_formula" in case:
        n = case["n"]
        i = np.arange(n, dtype=np.int64)
        a = (7 * i - 3).astype(np.int32)
        b = (0x7FFFFFFF - i).astype(np.int32)
        assert oracle.reduce_local(op, dt, a, b) == 0
        assert b[0] == case["expect_first"] and b[-1] == case["expect_last"]
        return
    if "in_f32_hex" in case:
        a, b = _f32(case["in_f32_hex"]), _f32(case["inout_f32_hex"])
        assert oracle.reduce_local(op, dt, a, b) == 0
        assert np.array_equal(b.view(np.uint32), _f32(case["expect_f32_hex"]).view(np.uint32))
        return
    if "inout_v_f32_hex" in case:
        a = np.zeros(1, dtype=np_dtype(kind))
        b = np.zeros(1, dtype=np_dtype(kind))
        a["v"], a["l"] = _f32(case["in_v_f32_hex"]), case["in_l"]
        b["v"], b["l"] = _f32(case["inout_v_f32_hex"]), case["inout_l"]
        assert oracle.reduce_local(op, dt, a, b) == 0
        assert b["v"].view(np.uint32)[0] == _f32(case["expect_v_f32_hex"]).view(np.uint32)[0]
        assert list(b["l"]) == case["expect_l"]
        return
    dtype = np_dtype(kind)
    if kind in ("ii",):
        a = np.array([tuple(x) for x in case["in"]], dtype=dtype)
        b = np.array([tuple(x) for x in case["inout"]], dtype=dtype)
        assert oracle.reduce_local(op, dt, a, b) == 0
        assert [list(x) for x in b.tolist()] == case["expect"]
        return
    if kind == "c8":
        a = np.array([complex(*x) for x in case["in"]], dtype=np.complex64)
        b = np.array([complex(*x) for x in case["inout"]], dtype=np.complex64)
        assert oracle.reduce_local(op, dt, a, b) == 0
        got = [["%.9g" % b[0].real, "%.9g" % b[0].imag]]
        assert got == case["expect_decimal9"]
        return
    a = np.array(case["in"], dtype=dtype)
    b = np.array(case["inout"], dtype=dtype)
    assert oracle.reduce_local(op, dt, a, b) == 0
    assert b.tolist() == case["expect"]


@pytest.mark.parametrize("pair", _kat()["illegal_pairs"], ids=lambda c: c["op"] + "_" + c["dt"])
def test_oracle_illegal_pairs(pair):
    assert oracle.op_check(h(pair["op"]), h(pair["dt"])) == pair["expect"]
    a = np.zeros(4, np.uint8)
    b = np.ones(4, np.uint8)
    assert oracle.reduce_local(h(pair["op"]), h(pair["dt"]), a, b) == pair["expect"]
    assert (b == 1).all()   # kernel not reached: inout untouched


def test_oracle_legality_matrix_shape():
    # SURVEY.md 8(a) notes: the legal (op, type) matrix
    legal = {op: {dt for dt in KIND if oracle.op_check(h(op), h(dt)) == 0} for op in OPS}
    cints = {d for d in KIND if KIND[d] in ("i1", "u1", "i2", "u2", "i4", "u4", "i8", "u8") and d not in (
        "MPI_INTEGER", "MPI_AINT", "MPI_OFFSET", "MPI_INTEGER1", "MPI_INTEGER2", "MPI_INTEGER4",
        "MPI_INTEGER8", "MPI_LOGICAL", "MPI_BYTE", "MPI_CHAR", "MPI_CHARACTER")}
    assert len(cints) == 18
    assert "MPI_BYTE" in legal["MPI_BAND"] and "MPI_BYTE" not in legal["MPI_SUM"]
    assert "MPI_C_BOOL" in legal["MPI_LXOR"] and "MPI_C_BOOL" not in legal["MPI_BXOR"]
    assert "MPI_LOGICAL" in legal["MPI_BOR"] and "MPI_LOGICAL" not in legal["MPI_MAX"]
    assert "MPI_FLOAT" in legal["MPI_LAND"] and "MPI_FLOAT" not in legal["MPI_BAND"]
    assert "MPI_COMPLEX" in legal["MPI_PROD"] and "MPI_COMPLEX" not in legal["MPI_MAX"]
    assert legal["MPI_MAXLOC"] == {d for d in KIND if KIND[d] in ("ii", "fi", "si", "di", "ff", "dd")}
    for op in OPS:
        assert cints <= legal[op] or op in ("MPI_MAXLOC", "MPI_MINLOC")
        for dt in NON_REDUCIBLE:
            assert oracle.op_check(h(op), h(dt)) == C.MPI_ERR_OP


def test_oracle_zero_count_and_wrap_types():
    rng = np.random.default_rng(1)
    for dt, kind in [("MPI_UNSIGNED_SHORT", "u2"), ("MPI_SHORT", "i2"), ("MPI_UINT64_T", "u8")]:
        a, b = gen(kind, "MPI_PROD", 257, rng), gen(kind, "MPI_PROD", 257, rng)
        exp = (a.astype(np.uint64) * b.astype(np.uint64)).astype(a.dtype) if kind != "u8" else a * b
        bb = b.copy()
        assert oracle.reduce_local(h("MPI_PROD"), h(dt), a, bb) == 0
        assert np.array_equal(bb, exp)


def _fold(op, xs):
    """tree ((x0 op x1) op (x2 op x3)) ... with numpy fp32 adds (left = inout)."""
    while len(xs) > 1:
        xs = [xs[i] + xs[i + 1] for i in range(0, len(xs), 2)]
    return xs[0]


@pytest.mark.parametrize("count", [64, 100003])   # RD (<=256 KiB) and Rabenseifner
def test_oracle_allreduce_tree_order_fp32(count):
    rng = np.random.default_rng(2)
    p = 8
    xs = [(rng.standard_normal(count) * 10.0 ** rng.integers(-6, 6, count)).astype(np.float32)
          for _ in range(p)]
    rb = [np.zeros(count, np.float32) for _ in range(p)]
    assert oracle.allreduce(C.MPI_SUM, C.MPI_FLOAT, xs, rb) == 0
    exp = _fold(None, list(xs))    # ((x0+x1)+(x2+x3))+((x4+x5)+(x6+x7))
    for r in range(p):
        assert np.array_equal(rb[r].view(np.uint32), exp.view(np.uint32))


def test_oracle_reduce_scatter_tree_order_fp32():
    rng = np.random.default_rng(3)
    p, n = 8, 100
    xs = [(rng.standard_normal(p * n) * 10.0 ** rng.integers(-6, 6, p * n)).astype(np.float32)
          for _ in range(p)]
    rb = [np.zeros(n, np.float32) for _ in range(p)]
    assert oracle.reduce_scatter(C.MPI_SUM, C.MPI_FLOAT, [n] * p, xs, rb) == 0   # 3200 B: halving
    # ((x0+x4)+(x2+x6))+((x1+x5)+(x3+x7)) for rank 0's block (SURVEY.md 8 notes)
    o = [xs[k][:n] for k in (0, 4, 2, 6, 1, 5, 3, 7)]
    assert np.array_equal(rb[0].view(np.uint32), _fold(None, o).view(np.uint32))


def test_oracle_reduce_scatter_pairwise_chain():
    rng = np.random.default_rng(4)
    p, n = 4, 40000                           # 640 KB >= 512 KiB: pairwise exchange
    xs = [rng.standard_normal(p * n).astype(np.float32) for _ in range(p)]
    rb = [np.zeros(n, np.float32) for _ in range(p)]
    assert oracle.reduce_scatter(C.MPI_SUM, C.MPI_FLOAT, [n] * p, xs, rb) == 0
    for r in range(p):
        acc = xs[r][r * n:(r + 1) * n].copy()
        for k in range(1, p):
            acc = acc + xs[(r - k) % p][r * n:(r + 1) * n]
        assert np.array_equal(rb[r], acc)


@pytest.mark.parametrize("p", [1, 2, 3, 5, 6, 7, 8])
def test_oracle_allreduce_integer_any_p(p):
    rng = np.random.default_rng(5 + p)
    for count in (10, 70000):
        xs = [rng.integers(-2**31, 2**31, count, dtype=np.int64).astype(np.int32) for _ in range(p)]
        rb = [np.zeros(count, np.int32) for _ in range(p)]
        assert oracle.allreduce(C.MPI_SUM, C.MPI_INT, xs, rb) == 0
        exp = np.sum(np.stack(xs).astype(np.int64), axis=0).astype(np.int32)   # wraps mod 2^32
        for r in range(p):
            assert np.array_equal(rb[r], exp)


def test_oracle_scan_association_fp32():
    # recursive-doubling scan (IscanBuildTaskList reduce.cpp:5285-5576): rank 5 of 8
    # ends with (x5+x4) + ((x1+x0) + (x3+x2)); Exscan rank 5: x4 + ((x1+x0) + (x3+x2))
    rng = np.random.default_rng(21)
    p, n = 8, 4096
    xs = [(rng.standard_normal(n) * 10.0 ** rng.integers(-6, 7, n)).astype(np.float32) for _ in range(p)]
    rb = [np.zeros(n, np.float32) for _ in range(p)]
    assert oracle.scan(C.MPI_SUM, C.MPI_FLOAT, xs, rb) == 0
    exp5 = (xs[5] + xs[4]) + ((xs[1] + xs[0]) + (xs[3] + xs[2]))
    assert np.array_equal(rb[5].view(np.uint32), exp5.view(np.uint32))
    ex = [np.full(n, 7.0, np.float32) for _ in range(p)]
    assert oracle.scan(C.MPI_SUM, C.MPI_FLOAT, xs, ex, exclusive=True) == 0
    assert np.array_equal(ex[5].view(np.uint32), (xs[4] + ((xs[1] + xs[0]) + (xs[3] + xs[2]))).view(np.uint32))
    assert (ex[0] == 7.0).all()          # rank 0's Exscan result is undefined: left untouched
    ints = [rng.integers(-2**31, 2**31, n, dtype=np.int64).astype(np.int32) for _ in range(5)]
    ri = [np.zeros(n, np.int32) for _ in range(5)]
    assert oracle.scan(C.MPI_SUM, C.MPI_INT, ints, ri) == 0
    cs = np.cumsum(np.stack(ints).astype(np.int64), axis=0).astype(np.int32)
    for r in range(5):
        assert np.array_equal(ri[r], cs[r])
