"""GPU: the non-blocking reductions follow the reference's NBC task lists.

MS-MPI builds MPI_Iallreduce / MPI_Ireduce / MPI_Ireduce_scatter[_block] from
task lists (reduce.cpp:1987-3257, 4346-4982, 6005-6768) that differ from the
blocking algorithms in two ways the results can show:
* the Rabenseifner gates of Iallreduce / Ireduce read the datatype's extent,
  the blocking calls MPI_Type_size: MPI_DOUBLE_INT (12 / 16 B) and
  MPI_SHORT_INT (6 / 8 B) switch algorithm at different counts, so MAXLOC /
  MINLOC with NaN values gives different per-rank results in the window;
* Ireduce's Rabenseifner folds and halves over root-relative ranks: fp32 SUM
  at a root other than 0 associates differently.
MSMPI_FORCE_ASYNC_WORKFLOW=1 makes the blocking calls take the NBC lists.

p ranks share the box's one GPU; every rank regenerates all inputs from a
seed and compares with the oracle's NBC (or blocking) simulation, bit for bit
(loc pairs: value and location fields; padding is pinned by test_gpu_local)."""
import os
import socket
import subprocess
import sys
import textwrap

import pytest

import msx

pytestmark = pytest.mark.gpu
REPO = msx.REPO_ROOT

WORKER = r'''
import ctypes, os, sys
sys.path.insert(0, os.path.join(REPO, "microsoft-mpi_amd")); sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import numpy as np, torch
import msx, oracle
from _cases import gen, KIND
C = msx.C
L = msx.init(errors_return=True)
r_, s_ = ctypes.c_int(), ctypes.c_int()
L.MPI_Comm_rank(C.MPI_COMM_WORLD, ctypes.byref(r_)); L.MPI_Comm_size(C.MPI_COMM_WORLD, ctypes.byref(s_))
rank, p = r_.value, s_.value
FORCE = os.environ.get("MSMPI_FORCE_ASYNC_WORKFLOW") == "1"
fails = []
checked = 0

def raw(a):
    return np.frombuffer(bytearray(a.tobytes()), dtype=a.dtype)

from _xfer import todev, fromdev   # page-locked transfers (tests/_xfer.py, DESIGN.md §2)

def dzeros(n):
    t = torch.zeros(max(n, 1), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    return t


def check(tag, got, exp):
    global checked
    checked += 1
    if exp.dtype.names:
        ok = all(np.ascontiguousarray(got[f]).tobytes() == np.ascontiguousarray(exp[f]).tobytes()
                 for f in exp.dtype.names)
    else:
        ok = got.tobytes() == exp.tobytes()
    if not ok:
        fails.append(tag)

def inputs(opn, dtn, count, seed):
    rng = np.random.default_rng(seed)
    return [raw(gen(KIND[dtn], opn, count, rng)) for _ in range(p)]

def wait(req):
    return L.MPI_Wait(ctypes.byref(req), ctypes.c_void_p(1))

# 1. allreduce on pair types inside the gate window: MPI_Iallreduce against the
# NBC list, MPI_Allreduce against the blocking algorithm (or the NBC list
# under MSMPI_FORCE_ASYNC_WORKFLOW)
for i, (opn, dtn, count) in enumerate([("MPI_MAXLOC", "MPI_DOUBLE_INT", 16400), ("MPI_MINLOC", "MPI_DOUBLE_INT", 21845),
                                       ("MPI_MAXLOC", "MPI_LONG_DOUBLE_INT", 20000),
                                       ("MPI_MAXLOC", "MPI_SHORT_INT", 40000), ("MPI_MINLOC", "MPI_SHORT_INT", 33000)]):
    op, dt = getattr(C, opn), getattr(C, dtn)
    xs = inputs(opn, dtn, count, 100 + i)
    e_nbc = [raw(np.zeros_like(x)) for x in xs]
    e_blk = [raw(np.zeros_like(x)) for x in xs]
    assert oracle.iallreduce(op, dt, xs, e_nbc) == 0
    assert oracle.allreduce(op, dt, xs, e_blk) == 0
    sb = todev(xs[rank])
    rb = dzeros(xs[rank].nbytes)
    req = ctypes.c_int()
    rc = L.MPI_Iallreduce(sb.data_ptr(), rb.data_ptr(), count, dt, op, C.MPI_COMM_WORLD, ctypes.byref(req))
    rc = rc or wait(req)
    if rc: fails.append(f"iallreduce {opn} {dtn} {count} rc={rc} {msx.last_error()}")
    else: check(f"iallreduce {opn} {dtn} {count}", fromdev(rb, xs[rank]), e_nbc[rank])
    rb2 = dzeros(xs[rank].nbytes)
    rc = L.MPI_Allreduce(sb.data_ptr(), rb2.data_ptr(), count, dt, op, C.MPI_COMM_WORLD)
    if rc: fails.append(f"allreduce {opn} {dtn} {count} rc={rc} {msx.last_error()}")
    else: check(f"allreduce {opn} {dtn} {count}", fromdev(rb2, xs[rank]), (e_nbc if FORCE else e_blk)[rank])
    # host buffers take the same schedule
    hb = raw(np.zeros_like(xs[rank]))
    rc = L.MPI_Iallreduce(xs[rank].ctypes.data, hb.ctypes.data, count, dt, op, C.MPI_COMM_WORLD, ctypes.byref(req))
    rc = rc or wait(req)
    if rc: fails.append(f"iallreduce host {opn} {dtn} rc={rc} {msx.last_error()}")
    else: check(f"iallreduce host {opn} {dtn} {count}", hb, e_nbc[rank])

# 2. MPI_Ireduce: pair types in the 64 KiB window and fp32 SUM at every root
# (root-relative Rabenseifner)
cases = [("MPI_MAXLOC", "MPI_DOUBLE_INT", 5000), ("MPI_MINLOC", "MPI_SHORT_INT", 12000),
         ("MPI_SUM", "MPI_FLOAT", 30001), ("MPI_SUM", "MPI_DOUBLE", 20000)]
for i, (opn, dtn, count) in enumerate(cases):
    op, dt = getattr(C, opn), getattr(C, dtn)
    xs = inputs(opn, dtn, count, 200 + i)
    roots = range(p) if opn == "MPI_SUM" else sorted({0, 1, p - 1})
    for root in roots:
        e_nbc = raw(np.zeros_like(xs[0]))
        e_blk = raw(np.zeros_like(xs[0]))
        assert oracle.ireduce(op, dt, root, xs, e_nbc) == 0
        assert oracle.reduce(op, dt, root, xs, e_blk) == 0
        sb = todev(xs[rank])
        rb = dzeros(xs[rank].nbytes)
        req = ctypes.c_int()
        rc = L.MPI_Ireduce(sb.data_ptr(), rb.data_ptr(), count, dt, op, root, C.MPI_COMM_WORLD, ctypes.byref(req))
        rc = rc or wait(req)
        if rc: fails.append(f"ireduce {opn} {dtn} root={root} rc={rc} {msx.last_error()}")
        elif rank == root: check(f"ireduce {opn} {dtn} {count} root={root}", fromdev(rb, xs[rank]), e_nbc)
        rb2 = dzeros(xs[rank].nbytes)
        rc = L.MPI_Reduce(sb.data_ptr(), rb2.data_ptr(), count, dt, op, root, C.MPI_COMM_WORLD)
        if rc: fails.append(f"reduce {opn} {dtn} root={root} rc={rc} {msx.last_error()}")
        elif rank == root: check(f"reduce {opn} {dtn} {count} root={root}", fromdev(rb2, xs[rank]),
                                 e_nbc if FORCE else e_blk)

# 3. MPI_Ireduce_scatter / _block, fp32 SUM: recursive halving (short) and
# pairwise (long), non-power-of-two p included; in place too
for i, per in enumerate((7, 3001, 70001)):
    counts = [per + (k % 3) for k in range(p)]
    xs = inputs("MPI_SUM", "MPI_FLOAT", sum(counts), 300 + i)
    ex = [raw(np.zeros(c, xs[0].dtype)) for c in counts]
    assert oracle.reduce_scatter(C.MPI_SUM, C.MPI_FLOAT, counts, xs, ex) == 0
    cnt = (ctypes.c_int * p)(*counts)
    sb = todev(xs[rank])
    rb = dzeros(counts[rank] * 4)
    req = ctypes.c_int()
    rc = L.MPI_Ireduce_scatter(sb.data_ptr(), rb.data_ptr(), cnt, C.MPI_FLOAT, C.MPI_SUM, C.MPI_COMM_WORLD,
                               ctypes.byref(req))
    rc = rc or wait(req)
    if rc: fails.append(f"ireduce_scatter {per} rc={rc} {msx.last_error()}")
    else: check(f"ireduce_scatter {per}", fromdev(rb, ex[rank], counts[rank]), ex[rank])
    ip = todev(xs[rank])
    rc = L.MPI_Ireduce_scatter(ctypes.c_void_p(-1 & 0xffffffffffffffff), ip.data_ptr(), cnt, C.MPI_FLOAT, C.MPI_SUM,
                               C.MPI_COMM_WORLD, ctypes.byref(req))
    rc = rc or wait(req)
    if rc: fails.append(f"ireduce_scatter in place {per} rc={rc} {msx.last_error()}")
    else: check(f"ireduce_scatter in place {per}", fromdev(ip, ex[rank], counts[rank]), ex[rank])
    xb = inputs("MPI_SUM", "MPI_FLOAT", per * p, 400 + i)
    eb = [raw(np.zeros(per, xb[0].dtype)) for _ in range(p)]
    assert oracle.reduce_scatter(C.MPI_SUM, C.MPI_FLOAT, [per] * p, xb, eb) == 0
    sbb, rbb = todev(xb[rank]), dzeros(per * 4)
    rc = L.MPI_Ireduce_scatter_block(sbb.data_ptr(), rbb.data_ptr(), per, C.MPI_FLOAT, C.MPI_SUM, C.MPI_COMM_WORLD,
                                     ctypes.byref(req))
    rc = rc or wait(req)
    if rc: fails.append(f"ireduce_scatter_block {per} rc={rc} {msx.last_error()}")
    else: check(f"ireduce_scatter_block {per}", fromdev(rbb, eb[rank]), eb[rank])

print("RESULT", rank, p, len(fails), checked, fails[:6], flush=True)
L.MPI_Finalize()
'''


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.parametrize("p,force", [(3, False), (5, False), (6, False), (2, False), (4, True), (3, True)])
def test_nbc_task_lists_on_one_gpu(p, force):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    port = _free_port()
    procs = []
    for r in range(p):
        env = dict(os.environ)
        env.update({"MSX_SIZE": str(p), "MSX_RANK": str(r), "MSX_DEVICE": "0",
                    "MSX_BOOTSTRAP_PORT": str(port), "MSX_BOOTSTRAP_ADDR": "127.0.0.1",
                    "MSX_BOOTSTRAP_TIMEOUT": "180"})
        if force:
            env["MSMPI_FORCE_ASYNC_WORKFLOW"] = "1"
        else:
            env.pop("MSMPI_FORCE_ASYNC_WORKFLOW", None)
        procs.append(subprocess.Popen([sys.executable, "-c", f"REPO={REPO!r}\n" + textwrap.dedent(WORKER)],
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env))
    results = []
    for pr in procs:
        try:
            o, e = pr.communicate(timeout=300)
        except subprocess.TimeoutExpired:
            pr.kill()
            o, e = pr.communicate()
        results.append((pr.returncode, o, e))
    for rc, o, e in results:
        assert rc == 0, (o + e)[-3000:]
        line = [l for l in o.splitlines() if l.startswith("RESULT")]
        assert line, (o + e)[-3000:]
        assert line[0].split()[3] == "0", line[0]
