"""CPU: the multi-rank path without a GPU.

1. The collective engine's schedules (expression trees per rank/block,
   msx_schedule_*) evaluated with the oracle's combine reproduce, bit for bit,
   the oracle's step-by-step simulation of the reference schedules
   (reduce.cpp:3768-4104, 917-1334) for p = 1..9, including the
   non-power-of-two fold and order-sensitive data (fp32 SUM over a wide
   dynamic range, MAX with NaN and +-0).
2. world_size-2 gloo: two processes exchange their contributions with
   torch.distributed (gloo) and each evaluates its own schedule; results match
   the simulator.
3. The library's own bootstrap (TCP hub): two MPI processes initialise, agree
   on rank/size, barrier, run a user-op MPI_Allreduce on host buffers (host
   code, no GPU), and fail loudly (MPI_ERR_OTHER) for builtin-op collectives
   on a GPU-less host instead of computing on the CPU.
"""
import ctypes
import json
import os
import socket
import subprocess
import sys
import textwrap

import numpy as np
import pytest

import msx
import oracle

C = msx.C
REPO = msx.REPO_ROOT


def schedule_tree(which, p, n):
    L = msx.lib()
    src = (ctypes.c_int * 32)()
    P, pm, ch = ctypes.c_int(), ctypes.c_uint(), ctypes.c_int()
    L.msx_schedule_tree.argtypes = [ctypes.c_int] * 3 + [ctypes.c_void_p] * 4
    assert L.msx_schedule_tree(which, p, n, src, ctypes.byref(P), ctypes.byref(pm), ctypes.byref(ch)) == 0
    return list(src), P.value, pm.value, bool(ch.value)


def schedule_block(p, count, n):
    L = msx.lib()
    s, ln = ctypes.c_int64(), ctypes.c_int64()
    L.msx_schedule_block.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    L.msx_schedule_block(p, count, n, ctypes.byref(s), ctypes.byref(ln))
    return s.value, ln.value


def algo(which, p, count, tsize):
    L = msx.lib()
    L.msx_schedule_algo.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int64, ctypes.c_int]
    return L.msx_schedule_algo(which, p, count, tsize)


def newrank(r, p):
    return msx.lib().msx_schedule_newrank(r, p)


def eval_tree(tree, xs, op, dt, lo, hi):
    """Evaluate a schedule tree with the oracle's combine (left = inout)."""
    src, P, pm, chain = tree
    if chain:
        v = xs[src[0]][lo:hi].copy()
        for k in range(1, P):
            oracle.reduce_local(op, dt, xs[src[k]][lo:hi].copy(), v)
        return v
    leaves = []
    for k in range(P):
        if src[2 * k] < 0:            # absent leaf (binomial tree over non-pof2 p)
            leaves.append(None)
            continue
        v = xs[src[2 * k]][lo:hi].copy()
        if (pm >> k) & 1:
            oracle.reduce_local(op, dt, xs[src[2 * k + 1]][lo:hi].copy(), v)
        leaves.append(v)
    w = 1
    while w < P:
        for k in range(0, P, 2 * w):
            if leaves[k + w] is not None:
                oracle.reduce_local(op, dt, leaves[k + w], leaves[k])
        w *= 2
    return leaves[0]


def engine_allreduce_result(xs, op, dt, rank):
    """What the engine computes for `rank` (recvbuf) from its schedules."""
    p, count = len(xs), xs[0].size
    esz = xs[0].dtype.itemsize
    n = newrank(rank, p)
    if algo(0, p, count, esz) == 0:        # recursive doubling: own lineage, whole vector
        nn = n if n >= 0 else newrank(rank + 1, p)
        return eval_tree(schedule_tree(0, p, nn), xs, op, dt, 0, count)
    out = np.empty_like(xs[0])
    pof2 = 1 << (p.bit_length() - 1)
    for m in range(pof2):                   # every block, computed by its owner m
        lo, ln = schedule_block(p, count, m)
        out[lo:lo + ln] = eval_tree(schedule_tree(0, p, m), xs, op, dt, lo, lo + ln)
    return out


def engine_reduce_result(xs, op, dt, root):
    """What the engine's MPI_Reduce leaves in root's recvbuf."""
    p, count = len(xs), xs[0].size
    if algo(2, p, count, xs[0].dtype.itemsize) == 4:                 # binomial
        return eval_tree(schedule_tree(4, p, root), xs, op, dt, 0, count)
    out = np.empty_like(xs[0])
    pof2 = 1 << (p.bit_length() - 1)
    for m in range(pof2):
        lo, ln = schedule_block(p, count, m)
        out[lo:lo + ln] = eval_tree(schedule_tree(3, p, m), xs, op, dt, lo, lo + ln)
    return out


def engine_reduce_scatter_result(xs, counts, op, dt, rank):
    p = len(xs)
    total = sum(counts)
    esz = xs[0].dtype.itemsize
    disp = np.concatenate([[0], np.cumsum(counts)]).astype(int)
    if algo(1, p, total, esz) == 3:
        t = schedule_tree(2, p, rank)
    else:
        n = newrank(rank, p)
        t = schedule_tree(1, p, n if n >= 0 else newrank(rank + 1, p))
    return eval_tree(t, xs, op, dt, disp[rank], disp[rank + 1])


def _data(p, count, op, seed):
    rng = np.random.default_rng(seed)
    xs = []
    for _ in range(p):
        if op == C.MPI_SUM:
            x = (rng.standard_normal(count) * 10.0 ** rng.integers(-6, 7, count)).astype(np.float32)
        else:
            x = rng.integers(-3, 4, count).astype(np.float32)
            x[rng.random(count) < 0.1] = np.nan
            x[rng.random(count) < 0.1] = -0.0
        xs.append(x)
    return xs


@pytest.mark.parametrize("p", [1, 2, 3, 4, 5, 6, 7, 8, 9])
@pytest.mark.parametrize("count", [13, 70001])      # recursive doubling / Rabenseifner
@pytest.mark.parametrize("opname", ["MPI_SUM", "MPI_MAX"])
def test_engine_allreduce_schedule_matches_reference_simulation(p, count, opname):
    op = getattr(C, opname)
    xs = _data(p, count, op, 100 * p + count % 97)
    rb = [np.zeros(count, np.float32) for _ in range(p)]
    assert oracle.allreduce(op, C.MPI_FLOAT, xs, rb) == 0
    for r in range(p):
        got = engine_allreduce_result(xs, op, C.MPI_FLOAT, r)
        assert np.array_equal(got.view(np.uint32), rb[r].view(np.uint32)), (p, count, r)


@pytest.mark.parametrize("p", [2, 3, 4, 5, 7, 8])
@pytest.mark.parametrize("per", [5, 9000])          # recursive halving / pairwise
@pytest.mark.parametrize("opname", ["MPI_SUM", "MPI_MAX"])
def test_engine_reduce_scatter_schedule_matches_reference_simulation(p, per, opname):
    op = getattr(C, opname)
    counts = [per + (i % 3) for i in range(p)]
    xs = _data(p, sum(counts), op, 7 * p + per)
    rb = [np.zeros(c, np.float32) for c in counts]
    assert oracle.reduce_scatter(op, C.MPI_FLOAT, counts, xs, rb) == 0
    for r in range(p):
        got = engine_reduce_scatter_result(xs, counts, op, C.MPI_FLOAT, r)
        assert np.array_equal(got.view(np.uint32), rb[r].view(np.uint32)), (p, per, r)


@pytest.mark.parametrize("p", [1, 2, 3, 5, 6, 7, 8, 9])
@pytest.mark.parametrize("count", [13, 30000])        # binomial / Rabenseifner (> 64 KiB)
@pytest.mark.parametrize("opname", ["MPI_SUM", "MPI_MAX"])
def test_engine_reduce_schedule_matches_reference_simulation(p, count, opname):
    op = getattr(C, opname)
    xs = _data(p, count, op, 31 * p + count % 89)
    for root in sorted({0, p - 1, p // 2}):
        exp = np.zeros(count, np.float32)
        assert oracle.reduce(op, C.MPI_FLOAT, root, xs, exp) == 0
        got = engine_reduce_result(xs, op, C.MPI_FLOAT, root)
        assert np.array_equal(got.view(np.uint32), exp.view(np.uint32)), (p, count, root)


def test_algorithm_gates_follow_reference_32bit_arithmetic():
    # allreduce: RD iff (unsigned)(count*size) <= 256 KiB or count < pof2 (reduce.cpp:3884)
    assert algo(0, 8, 65536, 4) == 0 and algo(0, 8, 65537, 4) == 1
    assert algo(0, 8, 7, 4) == 0
    assert algo(0, 8, 1 << 30, 4) == 0     # 4 GiB wraps to 0 bytes: recursive doubling
    # reduce_scatter: c4 (536870912 doubles = 2^32 B) wraps to 0 -> recursive halving
    assert algo(1, 8, 536870912, 8) == 2
    assert algo(1, 8, 65536, 8) == 3 and algo(1, 8, 65535, 8) == 2
    # reduce: Rabenseifner iff (unsigned)(count*size) > 64 KiB and count >= pof2 (reduce.cpp:151)
    assert algo(2, 8, 16384, 4) == 4 and algo(2, 8, 16385, 4) == 1


SWITCH_WORKER = r'''
import os, sys
sys.path.insert(0, os.path.join(REPO, "microsoft-mpi_amd")); sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import numpy as np
import msx, oracle
from test_collectives_cpu import (algo, engine_allreduce_result, engine_reduce_result,
                                  engine_reduce_scatter_result, _data)
C = msx.C
print("GATES", algo(0, 8, 64, 4), algo(0, 8, 70001, 4), algo(1, 8, 40, 4), algo(2, 8, 30000, 4), flush=True)
bad = []
for p in (3, 4, 8):
    for count in (13, 70001):
        xs = _data(p, count, C.MPI_SUM, 5 * p + count % 7)
        rb = [np.zeros(count, np.float32) for _ in range(p)]
        assert oracle.allreduce(C.MPI_SUM, C.MPI_FLOAT, xs, rb) == 0
        for r in range(p):
            if not np.array_equal(engine_allreduce_result(xs, C.MPI_SUM, C.MPI_FLOAT, r).view(np.uint32),
                                  rb[r].view(np.uint32)):
                bad.append(("allreduce", p, count, r))
        for root in (0, p - 1):
            exp = np.zeros(count, np.float32)
            assert oracle.reduce(C.MPI_SUM, C.MPI_FLOAT, root, xs, exp) == 0
            if not np.array_equal(engine_reduce_result(xs, C.MPI_SUM, C.MPI_FLOAT, root).view(np.uint32),
                                  exp.view(np.uint32)):
                bad.append(("reduce", p, count, root))
    for per in (5, 9000):
        counts = [per + (i % 3) for i in range(p)]
        xs = _data(p, sum(counts), C.MPI_SUM, 3 * p + per)
        rb = [np.zeros(c, np.float32) for c in counts]
        assert oracle.reduce_scatter(C.MPI_SUM, C.MPI_FLOAT, counts, xs, rb) == 0
        for r in range(p):
            if not np.array_equal(engine_reduce_scatter_result(xs, counts, C.MPI_SUM, C.MPI_FLOAT, r).view(np.uint32),
                                  rb[r].view(np.uint32)):
                bad.append(("reduce_scatter", p, per, r))
print("BAD", bad, flush=True)
'''


@pytest.mark.parametrize("env,gates", [
    # every switch point at 0: Rabenseifner from 8 floats on, pairwise reduce_scatter
    ({"MPICH_DEFAULT_ALLREDUCE_SHORT_MSG": "0", "MPICH_DEFAULT_REDUCE_SHORT_MSG": "0",
      "MPICH_DEFAULT_REDSCAT_COMMUTATIVE_LONG_MSG": "0"}, "1 1 3 1"),
    # huge: recursive doubling / binomial / recursive halving at every size
    ({"MPICH_DEFAULT_ALLREDUCE_SHORT_MSG": "2147483647", "MPICH_DEFAULT_REDUCE_SHORT_MSG": "999999999",
      "MPICH_DEFAULT_REDSCAT_COMMUTATIVE_LONG_MSG": "2000000000"}, "0 0 2 4"),
    # negative -> clamped to 0 (env_to_int's minval); 12 characters -> ignored (default);
    # 100 B: a 160-B reduce_scatter is already pairwise
    ({"MPICH_DEFAULT_ALLREDUCE_SHORT_MSG": "-5", "MPICH_DEFAULT_REDUCE_SHORT_MSG": "000000065536",
      "MPICH_DEFAULT_REDSCAT_COMMUTATIVE_LONG_MSG": "100"}, "1 1 3 1"),
])
def test_switch_points_follow_the_reference_environment(env, gates):
    """MPICH_DEFAULT_{ALLREDUCE,REDUCE}_SHORT_MSG / _REDSCAT_COMMUTATIVE_LONG_MSG
    move the flat algorithm switch points like mpid/env.cpp:514-608 (env_to_int:
    unset or over 11 characters -> default, clamped at 0); engine schedules and
    the oracle's step-by-step simulation (which reads the same variables) stay
    bit-identical on both sides of every moved gate."""
    e = dict(os.environ)
    e.update(env)
    pr = subprocess.run([sys.executable, "-c", f"REPO={REPO!r}\n" + textwrap.dedent(SWITCH_WORKER)],
                        capture_output=True, text=True, env=e, timeout=300)
    assert pr.returncode == 0, pr.stderr[-2000:]
    out = dict(l.split(" ", 1) for l in pr.stdout.splitlines() if l[:4] in ("GATE", "BAD "))
    assert out["GATES"] == gates, out
    assert out["BAD"] == "[]", out


# ---------------------------------------------------------------------------
# world_size 2 over gloo
# ---------------------------------------------------------------------------
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


GLOO_WORKER = r'''
import os, sys
sys.path.insert(0, os.path.join(REPO, "microsoft-mpi_amd")); sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import numpy as np, torch, torch.distributed as dist
import msx, oracle
from test_collectives_cpu import engine_allreduce_result, engine_reduce_scatter_result, _data
C = msx.C
dist.init_process_group("gloo", init_method="env://")
rank, p = dist.get_rank(), dist.get_world_size()
ok = True
for count in (33, 90001):
    for op in (C.MPI_SUM, C.MPI_MAX):
        mine = _data(p, count, op, 5 + count)[rank]
        bufs = [torch.zeros(count, dtype=torch.float32) for _ in range(p)]
        dist.all_gather(bufs, torch.from_numpy(mine))        # the exchange step over gloo
        xs = [b.numpy() for b in bufs]
        got = engine_allreduce_result(xs, op, C.MPI_FLOAT, rank)
        rb = [np.zeros(count, np.float32) for _ in range(p)]
        oracle.allreduce(op, C.MPI_FLOAT, xs, rb)
        ok &= np.array_equal(got.view(np.uint32), rb[rank].view(np.uint32))
        counts = [count // p] * p
        got = engine_reduce_scatter_result(xs, counts, op, C.MPI_FLOAT, rank)
        rs = [np.zeros(c, np.float32) for c in counts]
        oracle.reduce_scatter(op, C.MPI_FLOAT, counts, xs, rs)
        ok &= np.array_equal(got.view(np.uint32), rs[rank].view(np.uint32))
flag = torch.tensor([1 if ok else 0])
dist.all_reduce(flag, op=dist.ReduceOp.MIN)
print("RESULT", rank, int(flag.item()))
dist.destroy_process_group()
'''


def _spawn(code, ranks, extra_env):
    procs = []
    for r in range(ranks):
        env = dict(os.environ)
        env.update(extra_env(r))
        procs.append(subprocess.Popen([sys.executable, "-c", f"REPO={REPO!r}\n" + textwrap.dedent(code)],
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env))
    outs = []
    for pr in procs:
        try:
            o, e = pr.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            pr.kill()
            o, e = pr.communicate()
        outs.append((pr.returncode, o, e))
    return outs


def test_gloo_world_size_2_engine_schedule():
    port = _free_port()
    outs = _spawn(GLOO_WORKER, 2, lambda r: {"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port),
                                             "RANK": str(r), "WORLD_SIZE": "2"})
    for rc, o, e in outs:
        assert rc == 0, e[-2000:]
        assert "RESULT" in o and o.strip().split()[-1] == "1", o + e[-2000:]


MPI_WORKER = r'''
import ctypes, os, sys
sys.path.insert(0, os.path.join(REPO, "microsoft-mpi_amd"))
import numpy as np
import msx
C = msx.C
L = msx.init(errors_return=True)
r, s = ctypes.c_int(), ctypes.c_int()
L.MPI_Comm_rank(C.MPI_COMM_WORLD, ctypes.byref(r)); L.MPI_Comm_size(C.MPI_COMM_WORLD, ctypes.byref(s))
assert L.MPI_Barrier(C.MPI_COMM_WORLD) == 0
UF = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int))
def sub(a, b, n, dt):   # non-commutative: inout = in - inout
    x = np.ctypeslib.as_array((ctypes.c_double * n[0]).from_address(a))
    y = np.ctypeslib.as_array((ctypes.c_double * n[0]).from_address(b))
    y[:] = x - y
fn = UF(sub)
op = ctypes.c_int()
assert L.MPI_Op_create(fn, 0, ctypes.byref(op)) == 0
send = np.array([10.0 * (r.value + 1), 1.0 + r.value], dtype=np.float64)
recv = np.zeros(2, np.float64)
rc = L.MPI_Allreduce(send.ctypes.data, recv.ctypes.data, 2, C.MPI_DOUBLE, op.value, C.MPI_COMM_WORLD)
assert rc == 0, msx.last_error()
b = np.zeros(4, np.float32)
rc2 = L.MPI_Allreduce(b.ctypes.data, np.zeros(4, np.float32).ctypes.data, 4, C.MPI_FLOAT, C.MPI_SUM, C.MPI_COMM_WORLD)
gpu = L.msx_device_count() > 0
print("OUT", r.value, s.value, recv.tolist(), rc2, int(gpu))
assert L.MPI_Finalize() == 0
'''


def test_two_mpi_processes_bootstrap_and_user_op_allreduce():
    port = _free_port()
    outs = _spawn(MPI_WORKER, 2, lambda r: {"MSX_SIZE": "2", "MSX_RANK": str(r),
                                            "MSX_BOOTSTRAP_PORT": str(port), "MSX_BOOTSTRAP_ADDR": "127.0.0.1"})
    res = {}
    for rc, o, e in outs:
        assert rc == 0, e[-3000:]
        line = [l for l in o.splitlines() if l.startswith("OUT")][0].split(" ", 1)[1]
        rk, sz, rest = line.split(" ", 2)
        res[int(rk)] = (int(sz), rest)
    assert set(res) == {0, 1} and all(v[0] == 2 for v in res.values())
    # p = 2, recursive doubling with a non-commutative op: both ranks get
    # x0 op x1 = in(x0) - inout(x1) with the lower rank's data as `in`
    # (reduce.cpp:3909-3924): [10-20, 1-2] = [-10, -1]
    for rk in (0, 1):
        assert res[rk][1].startswith("[-10.0, -1.0]"), res
        gpu = res[rk][1].rstrip().endswith("1")
        rc2 = int(res[rk][1].split()[-2])
        assert rc2 == (0 if gpu else C.MPI_ERR_OTHER)


SCAN_WORKER = r'''
import ctypes, os, sys
sys.path.insert(0, os.path.join(REPO, "microsoft-mpi_amd"))
import numpy as np
import msx
C = msx.C
L = msx.init(errors_return=True)
r = ctypes.c_int()
L.MPI_Comm_rank(C.MPI_COMM_WORLD, ctypes.byref(r))
UF = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int))
def sub(a, b, n, dt):   # non-commutative, non-associative: inout = in - inout
    x = np.ctypeslib.as_array((ctypes.c_double * n[0]).from_address(a))
    y = np.ctypeslib.as_array((ctypes.c_double * n[0]).from_address(b))
    y[:] = x - y
fn = UF(sub)
op = ctypes.c_int()
assert L.MPI_Op_create(fn, 0, ctypes.byref(op)) == 0
for f in (L.MPI_Scan, L.MPI_Exscan):
    f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]
for f in (L.MPI_Iscan, L.MPI_Iexscan):
    f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                  ctypes.c_void_p]
send = np.array([10.0 * (r.value + 1)] * 3, dtype=np.float64)
inc, exc = np.zeros(3), np.full(3, 7.0)
assert L.MPI_Scan(send.ctypes.data, inc.ctypes.data, 3, C.MPI_DOUBLE, op.value, C.MPI_COMM_WORLD) == 0, msx.last_error()
assert L.MPI_Exscan(send.ctypes.data, exc.ctypes.data, 3, C.MPI_DOUBLE, op.value, C.MPI_COMM_WORLD) == 0
# non-blocking forms give the same results
inc2, exc2, req = np.zeros(3), np.full(3, 7.0), ctypes.c_int()
assert L.MPI_Iscan(send.ctypes.data, inc2.ctypes.data, 3, C.MPI_DOUBLE, op.value, C.MPI_COMM_WORLD, ctypes.byref(req)) == 0
assert L.MPI_Wait(ctypes.byref(req), ctypes.c_void_p(1)) == 0 and req.value == C.MPI_REQUEST_NULL
assert L.MPI_Iexscan(send.ctypes.data, exc2.ctypes.data, 3, C.MPI_DOUBLE, op.value, C.MPI_COMM_WORLD, ctypes.byref(req)) == 0
assert L.MPI_Wait(ctypes.byref(req), ctypes.c_void_p(1)) == 0
assert (inc2 == inc).all() and (exc2 == exc).all()
# MPI_Reduce with user ops: the reference's binomial tree (reduce.cpp:440-540)
opc = ctypes.c_int()
assert L.MPI_Op_create(fn, 1, ctypes.byref(opc)) == 0       # same function, flagged commutative
x2 = np.array([10.0 * 2 ** r.value], np.float64)
red = {}
for name, o in (("noncomm", op.value), ("comm", opc.value)):
    out = np.full(1, 7.0)
    assert L.MPI_Reduce(x2.ctypes.data, out.ctypes.data, 1, C.MPI_DOUBLE, o, 2, C.MPI_COMM_WORLD) == 0
    red[name] = out[0]
# MPI_Reduce_scatter_block with the commutative-flagged user op: recursive
# halving (32 B < 512 KiB), leaves x_{n ^ bitrev(k)}, left operand = inout
rs_in = np.array([10.0 * 2 ** r.value + j for j in range(4)], np.float64)
rs_out = np.zeros(1)
assert L.MPI_Reduce_scatter_block(rs_in.ctypes.data, rs_out.ctypes.data, 1, C.MPI_DOUBLE, opc.value,
                                  C.MPI_COMM_WORLD) == 0, msx.last_error()
red["rs"] = rs_out[0]
print("RED", r.value, red["noncomm"], red["comm"], red["rs"], flush=True)
import time
t0 = time.perf_counter()
for _ in range(500):                       # node-local shared-memory barrier
    assert L.MPI_Barrier(C.MPI_COMM_WORLD) == 0
print("BARRIER_US", (time.perf_counter() - t0) / 500 * 1e6, flush=True)
print("OUT", r.value, inc[0], exc[0], flush=True)
assert L.MPI_Finalize() == 0
'''


def test_four_mpi_processes_user_op_scan_follows_reference_task_order():
    """A non-associative user op exposes the recursive-doubling association of
    the reference's scan (IscanBuildTaskList, reduce.cpp:5285-5576): with
    x = [10, 20, 30, 40] and a op b = a - b, rank 3 gets (x0-x1)-(x2-x3) = 0
    (a sequential prefix would give -80) and Exscan rank 3 gets (x0-x1)-x2."""
    port = _free_port()
    outs = _spawn(SCAN_WORKER, 4, lambda r: {"MSX_SIZE": "4", "MSX_RANK": str(r),
                                             "MSX_BOOTSTRAP_PORT": str(port), "MSX_BOOTSTRAP_ADDR": "127.0.0.1"})
    got, red, rsv = {}, {}, {}
    for rc, o, e in outs:
        assert rc == 0, e[-3000:]
        _, rk, inc, exc = [l for l in o.splitlines() if l.startswith("OUT")][0].split()
        got[int(rk)] = (float(inc), float(exc))
        _, rk, nc, cm, rs = [l for l in o.splitlines() if l.startswith("RED")][0].split()
        red[int(rk)] = (float(nc), float(cm))
        rsv[int(rk)] = float(rs)
    # MPI_Reduce at root 2 of x = [10, 20, 40, 80] with a op b = a - b:
    # non-commutative -> tree rooted at 0: (x0-x1)-(x2-x3) = 30;
    # flagged commutative -> relative ranks from root 2: (x1-x0)-(x3-x2) = -30
    assert red[2] == (30.0, -30.0)
    assert all(red[k] == (7.0, 7.0) for k in (0, 1, 3))
    # reduce_scatter (recursive halving): rank 0 = (x3-x1)-(x2-x0) = 30 with
    # x = [10, 20, 40, 80]; rank 1 over x+1 with leaves [x1,x3,x0,x2] = -30
    assert rsv[0] == 30.0 and rsv[1] == -30.0
    assert [got[k][0] for k in range(4)] == [10.0, -10.0, -40.0, 0.0]
    assert [got[k][1] for k in range(4)] == [7.0, 10.0, -10.0, -40.0]


SPLIT_WORKER = r'''
import ctypes, os, sys
sys.path.insert(0, os.path.join(REPO, "microsoft-mpi_amd"))
import numpy as np
import msx
C = msx.C
L = msx.init(errors_return=True)
r = ctypes.c_int()
L.MPI_Comm_rank(C.MPI_COMM_WORLD, ctypes.byref(r))
rank = r.value
UF = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int))
def sub(a, b, n, dt):   # non-commutative: inout = in - inout
    x = np.ctypeslib.as_array((ctypes.c_double * n[0]).from_address(a))
    y = np.ctypeslib.as_array((ctypes.c_double * n[0]).from_address(b))
    y[:] = x - y
fn = UF(sub)
op = ctypes.c_int()
assert L.MPI_Op_create(fn, 0, ctypes.byref(op)) == 0
for f in (L.MPI_Allreduce, L.MPI_Scan):
    f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]
# split WORLD (5 ranks) by parity, keys reversing the order: odd = {3, 1},
# even = {4, 2, 0}; rank 4 is then rank 0 of the even group
sub_c = ctypes.c_int()
assert L.MPI_Comm_split(C.MPI_COMM_WORLD, rank % 2, -rank, ctypes.byref(sub_c)) == 0, msx.last_error()
sr, ss = ctypes.c_int(), ctypes.c_int()
L.MPI_Comm_rank(sub_c.value, ctypes.byref(sr)); L.MPI_Comm_size(sub_c.value, ctypes.byref(ss))
x = np.array([float(10 * (rank + 1))])
inc, out = np.zeros(1), np.zeros(1)
assert L.MPI_Scan(x.ctypes.data, inc.ctypes.data, 1, C.MPI_DOUBLE, op.value, sub_c.value) == 0, msx.last_error()
assert L.MPI_Allreduce(x.ctypes.data, out.ctypes.data, 1, C.MPI_DOUBLE, op.value, sub_c.value) == 0
# a duplicate of WORLD, and MPI_UNDEFINED -> MPI_COMM_NULL
dup, none = ctypes.c_int(), ctypes.c_int()
assert L.MPI_Comm_dup(C.MPI_COMM_WORLD, ctypes.byref(dup)) == 0
ds = ctypes.c_int(); L.MPI_Comm_size(dup.value, ctypes.byref(ds))
allw = np.zeros(1)
assert L.MPI_Allreduce(x.ctypes.data, allw.ctypes.data, 1, C.MPI_DOUBLE, op.value, dup.value) == 0
assert L.MPI_Comm_split(C.MPI_COMM_WORLD, 0 if rank == 2 else C.MPI_UNDEFINED, 0, ctypes.byref(none)) == 0
solo = none.value
if rank == 2:
    s1 = ctypes.c_int(); L.MPI_Comm_size(solo, ctypes.byref(s1)); assert s1.value == 1
    assert L.MPI_Comm_free(ctypes.byref(none)) == 0
else:
    assert solo == C.MPI_COMM_NULL
errs = [L.MPI_Comm_split(C.MPI_COMM_WORLD, -5, 0, ctypes.byref(none)),
        L.MPI_Comm_free(ctypes.byref(ctypes.c_int(C.MPI_COMM_WORLD)))]
assert L.MPI_Comm_free(ctypes.byref(sub_c)) == 0 and sub_c.value == C.MPI_COMM_NULL
assert L.MPI_Comm_free(ctypes.byref(dup)) == 0
print("OUT", rank, sr.value, ss.value, inc[0], out[0], ds.value, allw[0], errs[0], errs[1], flush=True)
assert L.MPI_Finalize() == 0
'''


def test_comm_split_dup_free_with_user_ops():
    """MPI_Comm_split / dup / free (api/mpi_comm.cpp): groups ordered by
    (key, rank), each with its own transport; a non-commutative user op pins
    the group order through the reference's scan and allreduce associations.
    The negative-color split is collective (all 5 ranks call it) and rejected
    on every rank before any exchange."""
    port = _free_port()
    outs = _spawn(SPLIT_WORKER, 5, lambda r: {"MSX_SIZE": "5", "MSX_RANK": str(r),
                                              "MSX_BOOTSTRAP_PORT": str(port), "MSX_BOOTSTRAP_ADDR": "127.0.0.1"})
    got = {}
    for rc, o, e in outs:
        assert rc == 0, e[-3000:]
        f = [l for l in o.splitlines() if l.startswith("OUT")][0].split()[1:]
        got[int(f[0])] = f[1:]
    x = {r: 10.0 * (r + 1) for r in range(5)}
    # even group in sub-rank order: world 4, 2, 0 (values 50, 30, 10); odd: 3, 1 (40, 20)
    exp_sub = {4: (0, 3), 2: (1, 3), 0: (2, 3), 3: (0, 2), 1: (1, 2)}
    for r in range(5):
        sr, ss = int(got[r][0]), int(got[r][1])
        assert (sr, ss) == exp_sub[r], (r, got[r])
    # scan, a op b = a - b, recursive doubling: sub-rank 1 -> y0 - y1, sub-rank 2 -> (y0 - y1) - y2
    assert float(got[4][2]) == 50.0 and float(got[2][2]) == 50.0 - 30.0 and float(got[0][2]) == (50.0 - 30.0) - 10.0
    assert float(got[3][2]) == 40.0 and float(got[1][2]) == 40.0 - 20.0
    # allreduce in the odd group (p = 2): y0 - y1 = 20 on both ranks
    assert float(got[3][3]) == 20.0 and float(got[1][3]) == 20.0
    for r in range(5):
        assert int(got[r][4]) == 5
        assert int(got[r][6]) == C.MPI_ERR_ARG and int(got[r][7]) == C.MPI_ERR_COMM
    # the duplicate of WORLD reduces like WORLD: every rank gets the same value
    assert len({got[r][5] for r in range(5)}) == 1


GROUP_WORKER = r'''
import ctypes, json, os, sys
sys.path.insert(0, os.path.join(REPO, "microsoft-mpi_amd"))
import msx
C = msx.C
L = msx.init(errors_return=True)
r = ctypes.c_int()
L.MPI_Comm_rank(C.MPI_COMM_WORLD, ctypes.byref(r))
rank = r.value
G = lambda: ctypes.c_int()
def members(g):
    n = ctypes.c_int(); assert L.MPI_Group_size(g, ctypes.byref(n)) == 0
    a = (ctypes.c_int * max(n.value, 1))(*range(n.value))
    w = G(); assert L.MPI_Comm_group(C.MPI_COMM_WORLD, ctypes.byref(w)) == 0
    out = (ctypes.c_int * max(n.value, 1))()
    assert L.MPI_Group_translate_ranks(g, n.value, a, w.value, out) == 0
    return list(out)[:n.value]
wg = G(); assert L.MPI_Comm_group(C.MPI_COMM_WORLD, ctypes.byref(wg)) == 0
ia = (ctypes.c_int * 3)(4, 1, 3)
inc = G(); assert L.MPI_Group_incl(wg.value, 3, ia, ctypes.byref(inc)) == 0
exc = G(); assert L.MPI_Group_excl(wg.value, 3, ia, ctypes.byref(exc)) == 0
rg = (ctypes.c_int * 6)(4, 0, -2, 1, 1, 1)          # ranges (4,0,-2) and (1,1,1): 4, 2, 0, 1
rinc = G(); assert L.MPI_Group_range_incl(wg.value, 2, rg, ctypes.byref(rinc)) == 0
rexc = G(); assert L.MPI_Group_range_excl(wg.value, 2, rg, ctypes.byref(rexc)) == 0
un = G(); assert L.MPI_Group_union(inc.value, rinc.value, ctypes.byref(un)) == 0
it = G(); assert L.MPI_Group_intersection(inc.value, rinc.value, ctypes.byref(it)) == 0
df = G(); assert L.MPI_Group_difference(rinc.value, inc.value, ctypes.byref(df)) == 0
gr = ctypes.c_int(); assert L.MPI_Group_rank(inc.value, ctypes.byref(gr)) == 0
cmp = []
for a, b in ((wg, wg), (inc, inc), (un, wg), (inc, rinc)):
    c = ctypes.c_int(); assert L.MPI_Group_compare(a.value, b.value, ctypes.byref(c)) == 0; cmp.append(c.value)
sim = (ctypes.c_int * 5)(4, 3, 2, 1, 0)
rv = G(); assert L.MPI_Group_incl(wg.value, 5, sim, ctypes.byref(rv)) == 0
c = ctypes.c_int(); assert L.MPI_Group_compare(rv.value, wg.value, ctypes.byref(c)) == 0; cmp.append(c.value)
# a split communicator's group holds WORLD process ids: odd = {3, 1} by key -rank
sub = ctypes.c_int()
assert L.MPI_Comm_split(C.MPI_COMM_WORLD, rank % 2, -rank, ctypes.byref(sub)) == 0
sg = G(); assert L.MPI_Comm_group(sub.value, ctypes.byref(sg)) == 0
# translate ranks incl. MPI_PROC_NULL and a non-member
tr_in = (ctypes.c_int * 3)(0, -1, 2)
tr_out = (ctypes.c_int * 3)()
assert L.MPI_Group_translate_ranks(inc.value, 3, tr_in, exc.value, tr_out) == 0
errs = [L.MPI_Group_incl(wg.value, 2, (ctypes.c_int * 2)(1, 1), ctypes.byref(G())),     # duplicate
        L.MPI_Group_incl(wg.value, 1, (ctypes.c_int * 1)(5), ctypes.byref(G())),        # out of range
        L.MPI_Group_range_incl(wg.value, 1, (ctypes.c_int * 3)(0, 4, 0), ctypes.byref(G())),   # stride 0
        L.MPI_Group_size(C.MPI_GROUP_NULL, ctypes.byref(ctypes.c_int())),
        L.MPI_Group_size(0x48000099, ctypes.byref(ctypes.c_int()))]
ex = ctypes.c_int(C.MPI_GROUP_EMPTY)
assert L.MPI_Group_free(ctypes.byref(ex)) == 0 and ex.value == C.MPI_GROUP_NULL
e0 = G(); assert L.MPI_Group_excl(wg.value, 0, None, ctypes.byref(e0)) == 0
print("M", rank, json.dumps([members(g.value) for g in (inc, exc, rinc, rexc, un, it, df, sg)]), flush=True)
# MPI_Comm_create: members of incl(4, 1, 3) get a communicator ranked in group
# order, the others MPI_COMM_NULL; a group reaching outside the communicator
# (WORLD's group on the parity sub-communicator) is MPI_ERR_GROUP on its members
cc = ctypes.c_int()
assert L.MPI_Comm_create(C.MPI_COMM_WORLD, inc.value, ctypes.byref(cc)) == 0
created = None
if cc.value != C.MPI_COMM_NULL:
    cr, cs, cg = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    L.MPI_Comm_rank(cc.value, ctypes.byref(cr)); L.MPI_Comm_size(cc.value, ctypes.byref(cs))
    assert L.MPI_Comm_group(cc.value, ctypes.byref(cg)) == 0
    rel = ctypes.c_int()
    assert L.MPI_Comm_compare(cc.value, C.MPI_COMM_WORLD, ctypes.byref(rel)) == 0
    created = [cr.value, cs.value, members(cg.value), rel.value]
    assert L.MPI_Group_free(ctypes.byref(cg)) == 0
    assert L.MPI_Comm_free(ctypes.byref(cc)) == 0
bad = ctypes.c_int()
create_err = L.MPI_Comm_create(sub.value, wg.value, ctypes.byref(bad))
print("G", rank, json.dumps([gr.value, cmp, list(tr_out), errs, created, create_err]), flush=True)
for g in (inc, exc, rinc, rexc, un, it, df, rv, sg, wg):
    assert L.MPI_Group_free(ctypes.byref(g)) == 0 and g.value == C.MPI_GROUP_NULL
assert L.MPI_Finalize() == 0
'''


def test_groups_five_processes():
    """MPI groups (api/mpi_group.cpp): incl / excl / range_incl / range_excl /
    union / intersection / difference member order, translate_ranks with
    MPI_PROC_NULL and non-members, compare (IDENT / SIMILAR / UNEQUAL), the
    reference's rank and range checks, groups of split communicators.
    Host-only calls: no GPU involved."""
    port = _free_port()
    outs = _spawn(GROUP_WORKER, 5, lambda r: {"MSX_SIZE": "5", "MSX_RANK": str(r),
                                              "MSX_BOOTSTRAP_PORT": str(port), "MSX_BOOTSTRAP_ADDR": "127.0.0.1"})
    U = -32766
    for rc, o, e in outs:
        assert rc == 0, e[-3000:]
        f = [l for l in o.splitlines() if l.startswith("G ")][0].split(" ", 2)
        rank = int(f[1])
        gr, cmp, tr, errs, created, create_err = json.loads(f[2])
        assert created == ({4: [0, 3, [4, 1, 3], C.MPI_UNEQUAL], 1: [1, 3, [4, 1, 3], C.MPI_UNEQUAL],
                            3: [2, 3, [4, 1, 3], C.MPI_UNEQUAL]}.get(rank)), (rank, created)
        assert create_err == C.MPI_ERR_GROUP
        # incl(4,1,3): rank of world 4 -> 0, 1 -> 1, 3 -> 2, others undefined
        assert gr == {4: 0, 1: 1, 3: 2}.get(rank, U), (rank, gr)
        # compare: world/world IDENT, inc/inc IDENT, union(inc, rinc) = 4,1,3,2,0 vs world SIMILAR,
        # inc vs rinc (sizes 3 / 4) UNEQUAL, reversed world SIMILAR
        assert list(cmp) == [C.MPI_IDENT, C.MPI_IDENT, C.MPI_SIMILAR, C.MPI_UNEQUAL, C.MPI_SIMILAR]
        # translate inc ranks (0 -> world 4, PROC_NULL, 2 -> world 3) into excl = {0, 2}
        assert list(tr) == [U, -1, U]
        assert list(errs) == [C.MPI_ERR_RANK, C.MPI_ERR_RANK, C.MPI_ERR_ARG, C.MPI_ERR_GROUP, C.MPI_ERR_GROUP]
        m = [l for l in o.splitlines() if l.startswith("M ")][0].split(" ", 2)[2]
        inc, exc, rinc, rexc, un, it, df, sg = json.loads(m)
        assert inc == [4, 1, 3] and exc == [0, 2] and rinc == [4, 2, 0, 1] and rexc == [3]
        assert un == [4, 1, 3, 2, 0] and it == [4, 1] and df == [2, 0]
        assert sg == ([3, 1] if rank % 2 else [4, 2, 0])


INTER_WORKER = r'''
import ctypes, json, os, sys
sys.path.insert(0, os.path.join(REPO, "microsoft-mpi_amd"))
import msx
C = msx.C
L = msx.init(errors_return=True)
r = ctypes.c_int()
L.MPI_Comm_rank(C.MPI_COMM_WORLD, ctypes.byref(r))
rank = r.value
W = C.MPI_COMM_WORLD
I = lambda: ctypes.c_int()
out = {}
def world_ranks(g):
    n = I(); L.MPI_Group_size(g, ctypes.byref(n))
    wg = I(); L.MPI_Comm_group(W, ctypes.byref(wg))
    a = (ctypes.c_int * max(n.value, 1))(*range(n.value)); o = (ctypes.c_int * max(n.value, 1))()
    L.MPI_Group_translate_ranks(g, n.value, a, wg.value, o)
    L.MPI_Group_free(ctypes.byref(wg))
    return list(o)[:n.value]
def members(comm):
    g = I(); L.MPI_Comm_group(comm, ctypes.byref(g)); m = world_ranks(g.value); L.MPI_Group_free(ctypes.byref(g)); return m

# A = {0, 1, 2}, B = {3, 4, 5}; B's leader is its local rank 1 (world 4)
loc = I()
assert L.MPI_Comm_split(W, 0 if rank < 3 else 1, rank, ctypes.byref(loc)) == 0
inA = rank < 3
ic = I()
rc = L.MPI_Intercomm_create(loc.value, 0 if inA else 1, W, 4 if inA else 0, 7, ctypes.byref(ic))
assert rc == 0, (rc, msx.last_error())
f, n, rs, lr = I(), I(), I(), I()
L.MPI_Comm_test_inter(ic.value, ctypes.byref(f)); L.MPI_Comm_size(ic.value, ctypes.byref(n))
L.MPI_Comm_remote_size(ic.value, ctypes.byref(rs)); L.MPI_Comm_rank(ic.value, ctypes.byref(lr))
rg = I(); assert L.MPI_Comm_remote_group(ic.value, ctypes.byref(rg)) == 0
out["inter"] = [f.value, n.value, rs.value, lr.value, world_ranks(rg.value), members(ic.value)]
L.MPI_Group_free(ctypes.byref(rg))
cmp = []
d = I(); assert L.MPI_Comm_dup(ic.value, ctypes.byref(d)) == 0
for a, b in ((ic.value, ic.value), (ic.value, d.value), (ic.value, W)):
    c = I(); L.MPI_Comm_compare(a, b, ctypes.byref(c)); cmp.append(c.value)
out["compare"] = cmp
L.MPI_Comm_test_inter(d.value, ctypes.byref(f)); out["dup_inter"] = f.value
assert L.MPI_Barrier(ic.value) == 0 and L.MPI_Barrier(d.value) == 0
# merges: A low, B high / both equal (rank 0's process id decides) / A high
merged = []
for ha, hb in ((0, 1), (0, 0), (1, 0)):
    m = I()
    assert L.MPI_Intercomm_merge(ic.value, ha if inA else hb, ctypes.byref(m)) == 0, msx.last_error()
    mr, ms = I(), I(); L.MPI_Comm_rank(m.value, ctypes.byref(mr)); L.MPI_Comm_size(m.value, ctypes.byref(ms))
    L.MPI_Comm_test_inter(m.value, ctypes.byref(f))
    merged.append([mr.value, ms.value, f.value, members(m.value)])
    assert L.MPI_Barrier(m.value) == 0
    L.MPI_Comm_free(ctypes.byref(m))
out["merge"] = merged
# inconsistent high within a group
m = I()
out["merge_notsame"] = L.MPI_Intercomm_merge(ic.value, 1 if rank in (0, 3) else 0, ctypes.byref(m))
buf = (ctypes.c_int * 4)()
errs = [L.MPI_Comm_remote_size(W, ctypes.byref(n)), L.MPI_Intercomm_merge(W, 0, ctypes.byref(m)),
        L.MPI_Scan(ctypes.c_void_p(ctypes.addressof(buf)), ctypes.c_void_p(ctypes.addressof(buf)), 0, C.MPI_INT,
                   C.MPI_SUM, ic.value),
        L.MPI_Win_create(ctypes.c_void_p(ctypes.addressof(buf)), 16, 4, C.MPI_INFO_NULL, ic.value, ctypes.byref(m)),
        L.MPI_Comm_split(ic.value, 0, 0, ctypes.byref(m)),
        L.MPI_Intercomm_create(loc.value, 7, W, 0, 1, ctypes.byref(m)),
        L.MPI_Allreduce(ctypes.c_void_p(-1), ctypes.c_void_p(ctypes.addressof(buf)), 4, C.MPI_INT, C.MPI_SUM, ic.value),
        L.MPI_Reduce(ctypes.c_void_p(ctypes.addressof(buf)), None, 4, C.MPI_INT, C.MPI_SUM, 3, ic.value),
        L.MPI_Reduce(ctypes.c_void_p(ctypes.addressof(buf)), None, 4, C.MPI_INT, C.MPI_SUM, C.MPI_PROC_NULL, ic.value)]
out["errs"] = errs
# a second pair of intercommunicators through a peer communicator that does
# not contain every process: P = {0..3} -> {0,1} x {2,3}; Q = {4,5} -> {4} x {5}
pq = I(); assert L.MPI_Comm_split(W, 0 if rank < 4 else 1, rank, ctypes.byref(pq)) == 0
pr = I(); L.MPI_Comm_rank(pq.value, ctypes.byref(pr))
half = I()
if rank < 4:
    assert L.MPI_Comm_split(pq.value, pr.value // 2, pr.value, ctypes.byref(half)) == 0
    remote = 2 if pr.value < 2 else 0
else:
    assert L.MPI_Comm_split(pq.value, pr.value, 0, ctypes.byref(half)) == 0
    remote = 1 - pr.value
ic2 = I()
assert L.MPI_Intercomm_create(half.value, 0, pq.value, remote, 11, ctypes.byref(ic2)) == 0, msx.last_error()
g2 = I(); L.MPI_Comm_remote_group(ic2.value, ctypes.byref(g2))
out["ic2_remote"] = world_ranks(g2.value)
L.MPI_Group_free(ctypes.byref(g2))
for c in (ic2, half, pq, d, ic, loc):
    assert L.MPI_Comm_free(ctypes.byref(c)) == 0 and c.value == C.MPI_COMM_NULL
print("J", rank, json.dumps(out), flush=True)
assert L.MPI_Finalize() == 0
'''


def test_intercommunicators_six_processes():
    """MPI_Intercomm_create (api/mpi_comm.cpp:1482-1610: leaders exchange the
    groups, here over the world mailbox; a peer communicator that does not
    contain every process), MPI_Comm_remote_size / remote_group /
    test_inter, MPI_Comm_compare on intercommunicators (api/mpi_comm.cpp:82-134),
    MPI_Comm_dup, MPI_Barrier over both groups, MPI_Intercomm_merge ordering
    (:1680-1830: high = false first; equal high -> the group whose rank 0 has
    the lower process id first; **notsame), and the intracommunicator-only
    checks.  No GPU: creation and synchronisation only."""
    port = _free_port()
    outs = _spawn(INTER_WORKER, 6, lambda r: {"MSX_SIZE": "6", "MSX_RANK": str(r), "MSX_BOOTSTRAP_PORT": str(port),
                                             "MSX_BOOTSTRAP_ADDR": "127.0.0.1"})
    for rc, o, e in outs:
        assert rc == 0, (o + e)[-3000:]
        line = [l for l in o.splitlines() if l.startswith("J ")][0].split(" ", 2)
        rank, d = int(line[1]), json.loads(line[2])
        A, B = [0, 1, 2], [3, 4, 5]
        inA = rank < 3
        assert d["inter"] == [1, 3, 3, rank % 3, B if inA else A, A if inA else B]
        assert d["compare"] == [C.MPI_IDENT, C.MPI_CONGRUENT, C.MPI_UNEQUAL]
        assert d["dup_inter"] == 1
        m01, m00, m10 = d["merge"]
        assert m01 == [rank, 6, 0, list(range(6))]
        assert m00 == [rank, 6, 0, list(range(6))]
        assert m10 == [(rank + 3) % 6, 6, 0, B + A]
        assert d["merge_notsame"] == C.MPI_ERR_ARG
        # remote_size / merge of an intracommunicator, scan / window / split of an
        # intercommunicator, a local leader out of range, MPI_IN_PLACE allreduce
        # on an intercommunicator, a root outside the remote group, MPI_PROC_NULL
        assert d["errs"] == [C.MPI_ERR_COMM, C.MPI_ERR_COMM, C.MPI_ERR_COMM, C.MPI_ERR_COMM, C.MPI_ERR_COMM,
                             C.MPI_ERR_RANK, C.MPI_ERR_BUFFER, C.MPI_ERR_ROOT, C.MPI_SUCCESS]
        assert d["ic2_remote"] == {0: [2, 3], 1: [2, 3], 2: [0, 1], 3: [0, 1], 4: [5], 5: [4]}[rank]


@pytest.mark.parametrize("p", [2, 3, 5, 6, 7, 8, 9, 16, 32])
def test_two_step_chunk_plan_covers_and_keeps_owners(p):
    """The pipelined two-step allreduce's chunk plan (msx_schedule_two_step,
    the function do_allreduce itself runs): over all ranks and chunks the
    ranges cover [0, count) exactly once, and each lies inside the block of
    the owner it is evaluated with (reduce.cpp:3927-4066's block of newrank
    `owner`) -- so cutting a message into chunks changes the work split, never
    the tree an element gets."""
    import msx
    L = msx.lib()
    i64 = ctypes.c_int64
    for esz in (4, 8):
        ce = i64()
        L.msx_schedule_two_step(p, 1000, esz, 0, ctypes.byref(ce), (i64 * 3)(), 1)
        pc = ce.value
        assert pc > 0 and pc % (p * 16) == 0
        for count in (p, 1001, 300001, pc - 1, pc, pc + 1, 3 * pc + 12345):
            cover = []
            for r in range(p):
                cap = 4096
                out = (i64 * (3 * cap))()
                n = L.msx_schedule_two_step(p, count, esz, r, ctypes.byref(ce), out, cap)
                assert n >= 0
                for k in range(n):
                    e0, e1, owner = out[3 * k], out[3 * k + 1], out[3 * k + 2]
                    assert 0 <= e0 < e1 <= count
                    st, ln = i64(), i64()
                    L.msx_schedule_block(p, count, owner, ctypes.byref(st), ctypes.byref(ln))
                    assert st.value <= e0 and e1 <= st.value + ln.value, (p, count, r, e0, e1, owner)
                    cover.append((e0, e1))
            cover.sort()
            assert cover[0][0] == 0 and cover[-1][1] == count
            assert all(a[1] == b[0] for a, b in zip(cover, cover[1:])), (p, count)
