"""CPU: the reference's NBC task lists (MPI_Iallreduce / MPI_Ireduce /
MPI_Ireduce_scatter, and the blocking calls under MSMPI_FORCE_ASYNC_WORKFLOW)
against its blocking schedules.

Where they differ (reduce.cpp):
* the Rabenseifner gates of IallreduceBuildTaskList (:4717, :4791, :4881) and
  IreduceBuildTaskList (:6701, :6740) multiply the count by the datatype's
  EXTENT, the blocking calls (:151, :3884) and both reduce_scatter forms
  (:1705, :3201) by MPI_Type_size.  For the pair types the two differ
  (MPI_DOUBLE_INT / MPI_LONG_DOUBLE_INT 16 vs 12 bytes, MPI_SHORT_INT 8 vs 6,
  datatype.cpp:1282-1293), so a window of counts takes different algorithms;
* IreduceBuildScatterGatherTaskList (:6267-6670) folds and halves over ranks
  RELATIVE TO THE ROOT, the blocking Rabenseifner reduce over absolute ranks
  (:174-300): for a root other than 0 the fp association differs.

Each test evaluates the engine's own schedule (msx_schedule_algo_dt, the trees)
with the oracle's combine and compares with the oracle's step-by-step NBC
simulation (oracle_iallreduce / oracle_ireduce), bit for bit."""
import numpy as np
import pytest

import msx
import oracle
from _cases import gen, np_dtype
from test_collectives_cpu import _data, eval_tree, newrank, schedule_block, schedule_tree

import ctypes

C = msx.C


def algo_dt(which, p, count, dt, nbc):
    L = msx.lib()
    L.msx_schedule_algo_dt.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int64, ctypes.c_int, ctypes.c_int]
    return L.msx_schedule_algo_dt(which, p, count, dt, 1 if nbc else 0)


def ireduce_tree(p, n, root):
    L = msx.lib()
    src = (ctypes.c_int * 32)()
    P, pm, ch = ctypes.c_int(), ctypes.c_uint(), ctypes.c_int()
    L.msx_schedule_ireduce_tree.argtypes = [ctypes.c_int] * 3 + [ctypes.c_void_p] * 4
    assert L.msx_schedule_ireduce_tree(p, n, root, src, ctypes.byref(P), ctypes.byref(pm), ctypes.byref(ch)) == 0
    return list(src), P.value, pm.value, bool(ch.value)


def engine_allreduce(xs, op, dt, rank, nbc):
    p, count = len(xs), xs[0].size
    if algo_dt(0, p, count, dt, nbc) == 0:            # recursive doubling, own lineage
        n = newrank(rank, p)
        return eval_tree(schedule_tree(0, p, n if n >= 0 else newrank(rank + 1, p)), xs, op, dt, 0, count)
    out = np.empty_like(xs[0])
    pof2 = 1 << (p.bit_length() - 1)
    for m in range(pof2):
        lo, ln = schedule_block(p, count, m)
        out[lo:lo + ln] = eval_tree(schedule_tree(0, p, m), xs, op, dt, lo, lo + ln)
    return out


def engine_reduce(xs, op, dt, root, nbc):
    p, count = len(xs), xs[0].size
    if algo_dt(2, p, count, dt, nbc) == 4:            # binomial (identical in both forms)
        return eval_tree(schedule_tree(4, p, root), xs, op, dt, 0, count)
    out = np.empty_like(xs[0])
    pof2 = 1 << (p.bit_length() - 1)
    for m in range(pof2):
        lo, ln = schedule_block(p, count, m)
        t = ireduce_tree(p, m, root) if nbc else schedule_tree(3, p, m)
        out[lo:lo + ln] = eval_tree(t, xs, op, dt, lo, lo + ln)
    return out


def same_bytes(a, b):
    """Bitwise equality of the data: every field of a pair type (numpy copies
    structured records field by field, so padding is not compared here; the
    GPU tests pin padding preservation)."""
    if a.dtype.names:
        return all(np.array_equal(np.ascontiguousarray(a[f]).view(np.uint8), np.ascontiguousarray(b[f]).view(np.uint8))
                   for f in a.dtype.names)
    return np.array_equal(a.view(np.uint8), b.view(np.uint8))


def _pairs(kind, p, count, seed):
    """Loc-pair inputs with NaN values and many ties (the MAXLOC/MINLOC cases
    whose per-rank results depend on the schedule); padding bytes random."""
    rng = np.random.default_rng(seed)
    xs = []
    for _ in range(p):
        a = gen(kind, "MPI_MAXLOC", count, rng)
        raw = a.view(np.uint8).reshape(count, -1)
        pad = rng.integers(0, 256, raw.shape, dtype=np.uint8)
        dt = np_dtype(kind)
        mask = np.ones(dt.itemsize, bool)                    # padding = bytes outside the fields
        for name in dt.names:
            off = dt.fields[name][1]
            mask[off:off + dt.fields[name][0].itemsize] = False
        raw[:, mask] = pad[:, mask]
        xs.append(a)
    return xs


# ---------------------------------------------------------------------------
# the gates
# ---------------------------------------------------------------------------
def test_type_size_and_extent_of_the_pair_types(msxlib):
    """MPI_Type_size vs extent as the reference builds the pair types."""
    L = msxlib
    for name, size, extent in [("MPI_DOUBLE_INT", 12, 16), ("MPI_LONG_DOUBLE_INT", 12, 16),
                               ("MPI_SHORT_INT", 6, 8), ("MPI_FLOAT_INT", 8, 8), ("MPI_2INT", 8, 8),
                               ("MPI_LONG_INT", 8, 8), ("MPI_2REAL", 8, 8), ("MPI_2DOUBLE_PRECISION", 16, 16)]:
        dt = getattr(C, name)
        assert oracle.type_size(dt) == size, name
        assert oracle.kind_size(dt) == extent, name
        s = ctypes.c_int()
        assert L.MPI_Type_size(dt, ctypes.byref(s)) == 0 and s.value == size, name
        lb, ext = ctypes.c_int64(), ctypes.c_int64()
        assert L.MPI_Type_get_extent(dt, ctypes.byref(lb), ctypes.byref(ext)) == 0 and ext.value == extent, name


def test_nbc_and_blocking_gates_diverge_for_pair_types():
    """Allreduce (short 256 KiB): MPI_DOUBLE_INT counts 16385..21845 are
    Rabenseifner for the NBC task list (16 B each) but recursive doubling for
    the blocking call (12 B each); MPI_SHORT_INT 32769..43690 likewise (8 / 6 B).
    Reduce (short 64 KiB): MPI_DOUBLE_INT 4097..5461."""
    DI, SI, F = C.MPI_DOUBLE_INT, C.MPI_SHORT_INT, C.MPI_FLOAT
    for c in (16385, 20000, 21845):
        assert algo_dt(0, 8, c, DI, True) == 1 and algo_dt(0, 8, c, DI, False) == 0, c
        assert algo_dt(0, 8, c, C.MPI_LONG_DOUBLE_INT, True) == 1
        assert algo_dt(0, 8, c, C.MPI_LONG_DOUBLE_INT, False) == 0
    assert algo_dt(0, 8, 16384, DI, True) == 0 and algo_dt(0, 8, 21846, DI, False) == 1
    for c in (32769, 43690):
        assert algo_dt(0, 8, c, SI, True) == 1 and algo_dt(0, 8, c, SI, False) == 0, c
    for c in (4097, 5461):
        assert algo_dt(2, 8, c, DI, True) == 1 and algo_dt(2, 8, c, DI, False) == 4, c
    assert algo_dt(2, 8, 5462, DI, False) == 1 and algo_dt(2, 8, 4096, DI, True) == 4
    # types whose size equals their extent gate alike
    for c in (65536, 65537):
        assert algo_dt(0, 8, c, F, True) == algo_dt(0, 8, c, F, False)
    # reduce_scatter gates on MPI_Type_size in both forms (:1705, :3201)
    assert algo_dt(1, 8, 43690, DI, True) == 2 and algo_dt(1, 8, 43691, DI, True) == 3
    assert algo_dt(1, 8, 43691, DI, False) == 3
    # the 32-bit wrap: 268435456 DOUBLE_INTs = 2^32 B of extent -> 0 -> recursive
    # doubling for the NBC call; 12 * 268435456 wraps to 2^31 > 256 KiB -> Rabenseifner
    assert algo_dt(0, 8, 268435456, DI, True) == 0 and algo_dt(0, 8, 268435456, DI, False) == 1


# ---------------------------------------------------------------------------
# engine schedules vs the oracle's NBC simulation
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("p", [2, 3, 4, 5, 6, 8])
@pytest.mark.parametrize("kind,dtname,count", [("di", "MPI_DOUBLE_INT", 16400), ("di", "MPI_DOUBLE_INT", 21845),
                                               ("si", "MPI_SHORT_INT", 40000)])
@pytest.mark.parametrize("opname", ["MPI_MAXLOC", "MPI_MINLOC"])
def test_iallreduce_pair_types_in_the_gate_window(p, kind, dtname, count, opname):
    """Counts where the NBC and blocking gates pick different algorithms: the
    engine's NBC schedule reproduces oracle_iallreduce and its blocking
    schedule oracle_allreduce, every rank, every field bit for bit."""
    op, dt = getattr(C, opname), getattr(C, dtname)
    xs = _pairs(kind, p, count, 11 * p + count)
    for nbc, sim in ((True, oracle.iallreduce), (False, oracle.allreduce)):
        rb = [np.zeros(count, xs[0].dtype) for _ in range(p)]
        assert sim(op, dt, xs, rb) == 0
        for r in range(p):
            assert same_bytes(engine_allreduce(xs, op, dt, r, nbc), rb[r]), (nbc, p, count, r)


def test_nbc_and_blocking_results_differ_in_the_window():
    """The distinction is observable: MAXLOC with NaN values gives different
    per-rank results under the two schedules in the gate window (p = 3)."""
    p, count = 3, 20000
    xs = _pairs("di", p, count, 4242)
    a = [np.zeros(count, xs[0].dtype) for _ in range(p)]
    b = [np.zeros(count, xs[0].dtype) for _ in range(p)]
    assert oracle.iallreduce(C.MPI_MAXLOC, C.MPI_DOUBLE_INT, xs, a) == 0
    assert oracle.allreduce(C.MPI_MAXLOC, C.MPI_DOUBLE_INT, xs, b) == 0
    assert any(not same_bytes(a[r], b[r]) for r in range(p))


@pytest.mark.parametrize("p", [2, 3, 5, 6, 7, 8])
@pytest.mark.parametrize("kind,dtname,count", [("di", "MPI_DOUBLE_INT", 5000), ("si", "MPI_SHORT_INT", 12000)])
@pytest.mark.parametrize("opname", ["MPI_MAXLOC", "MPI_MINLOC"])
def test_ireduce_pair_types_in_the_gate_window(p, kind, dtname, count, opname):
    op, dt = getattr(C, opname), getattr(C, dtname)
    xs = _pairs(kind, p, count, 13 * p + count)
    for root in sorted({0, 1, p - 1}):
        for nbc, sim in ((True, oracle.ireduce), (False, oracle.reduce)):
            exp = np.zeros(count, xs[0].dtype)
            assert sim(op, dt, root, xs, exp) == 0
            assert same_bytes(engine_reduce(xs, op, dt, root, nbc), exp), (nbc, p, root)


@pytest.mark.parametrize("p", [2, 3, 4, 5, 6, 7, 8, 9])
@pytest.mark.parametrize("count", [13, 30000])
def test_ireduce_fp32_sum_root_relative_tree(p, count):
    """fp32 SUM over a wide dynamic range: the root-relative Rabenseifner of
    MPI_Ireduce is reproduced for every root, and (for count 30000, p >= 3)
    differs from the blocking tree for some root."""
    xs = _data(p, count, C.MPI_SUM, 17 * p + count)
    differs = False
    for root in range(p):
        exp_nbc = np.zeros(count, np.float32)
        exp_blk = np.zeros(count, np.float32)
        assert oracle.ireduce(C.MPI_SUM, C.MPI_FLOAT, root, xs, exp_nbc) == 0
        assert oracle.reduce(C.MPI_SUM, C.MPI_FLOAT, root, xs, exp_blk) == 0
        got = engine_reduce(xs, C.MPI_SUM, C.MPI_FLOAT, root, True)
        assert np.array_equal(got.view(np.uint32), exp_nbc.view(np.uint32)), (p, count, root)
        got = engine_reduce(xs, C.MPI_SUM, C.MPI_FLOAT, root, False)
        assert np.array_equal(got.view(np.uint32), exp_blk.view(np.uint32)), (p, count, root)
        differs |= not np.array_equal(exp_nbc.view(np.uint32), exp_blk.view(np.uint32))
        if root == 0:   # relative == absolute ranks
            assert np.array_equal(exp_nbc.view(np.uint32), exp_blk.view(np.uint32))
    if count == 30000 and p >= 3:
        assert differs, p


@pytest.mark.parametrize("p", [3, 5, 6])
@pytest.mark.parametrize("per", [5, 9000])
def test_ireduce_scatter_fp32_sum_non_pof2(p, per):
    """MPI_Ireduce_scatter's task lists (short: recursive halving with the
    odd-keeps fold, :1987-2406; long: pairwise, :2412-2676) give the blocking
    results; the engine runs that one schedule for both."""
    counts = [per + (i % 3) for i in range(p)]
    xs = _data(p, sum(counts), C.MPI_SUM, 23 * p + per)
    rb = [np.zeros(c, np.float32) for c in counts]
    assert oracle.reduce_scatter(C.MPI_SUM, C.MPI_FLOAT, counts, xs, rb) == 0
    from test_collectives_cpu import engine_reduce_scatter_result
    for r in range(p):
        got = engine_reduce_scatter_result(xs, counts, C.MPI_SUM, C.MPI_FLOAT, r)
        assert np.array_equal(got.view(np.uint32), rb[r].view(np.uint32)), (p, per, r)
