"""GPU, >= 2 GPUs: MSX_TRANSPORT=rccl_native -- this library's MPI reductions on
RCCL's own collectives: ncclAllReduce / ncclReduce /
ncclReduceScatter where the (op, type) pair maps onto RCCL's, the reference's
trees (RCCL send/recv plane) everywhere else.

RCCL associates in its own ring/tree order, so the checks are the ones §8(d)
states for that mode: integer ops and MAX/MIN without NaN bit-exact against the
oracle; fp32 / fp64 SUM within |y - y_ref| <= 2 (p-1) eps sum_r |x_r| per
element (eps = 2^-24 / 2^-53); pairs RCCL lacks (BAND, MAXLOC, ragged
reduce_scatter) bit-exact, since they keep the reference order.  One rank per
GPU; the one-GPU box skips (RCCL refuses two ranks on one GPU), the driver's
multi-GPU node runs it.  The shared-GPU fallback of the same setting is in
test_gpu_multirank.py (rccl_native case)."""
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
torch.cuda.set_device(int(os.environ["MSX_DEVICE"]))
fails, checked = [], 0
IN_PLACE = ctypes.c_void_p(-1 & 0xffffffffffffffff)

def raw(a):
    return np.frombuffer(bytearray(a.tobytes()), dtype=a.dtype)

from _xfer import todev, fromdev   # page-locked transfers (tests/_xfer.py, DESIGN.md §2)

def dzeros(n):
    t = torch.zeros(max(n, 1), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    return t


def inputs(opn, dtn, count, seed):
    rng = np.random.default_rng(seed)
    return [raw(gen(KIND[dtn], opn, count, rng)) for _ in range(p)]

def check(tag, got, exp, xs=None):
    global checked
    checked += 1
    if xs is None or got.dtype.names or got.dtype.kind not in "f":
        if exp.dtype.names:
            ok = all(np.ascontiguousarray(got[f]).tobytes() == np.ascontiguousarray(exp[f]).tobytes()
                     for f in exp.dtype.names)
        else:
            ok = got.tobytes() == exp.tobytes()
    else:
        eps = 2.0 ** -24 if got.dtype == np.float32 else 2.0 ** -53
        bound = 2 * (p - 1) * eps * np.sum([np.abs(x.astype(np.float64)) for x in xs], axis=0)
        ok = bool(np.all(np.abs(got.astype(np.float64) - exp.astype(np.float64)) <= bound))
    if not ok:
        fails.append(tag)

# allreduce: mapped pairs (RCCL order) and unmapped ones (reference order)
for i, (opn, dtn, count, tol) in enumerate([("MPI_SUM", "MPI_INT", 300001, False), ("MPI_SUM", "MPI_FLOAT", 1 << 20, True),
                                            ("MPI_SUM", "MPI_DOUBLE", 100003, True), ("MPI_MAX", "MPI_DOUBLE", 70001, False),
                                            ("MPI_MIN", "MPI_UNSIGNED_CHAR", 5000, False), ("MPI_PROD", "MPI_INT64_T", 4099, False),
                                            ("MPI_BAND", "MPI_UINT64_T", 65536, False),
                                            ("MPI_MAXLOC", "MPI_DOUBLE_INT", 40000, False)]):
    op, dt = getattr(C, opn), getattr(C, dtn)
    xs = inputs(opn, dtn, count, 100 + i)
    if tol:           # finite data: inf - inf, overflow and NaN payloads depend on the order
        rng = np.random.default_rng(100 + i)
        xs = [raw(rng.uniform(-1, 1, count).astype(xs[0].dtype)) for _ in range(p)]
    elif opn in ("MPI_MAX", "MPI_MIN") and xs[0].dtype.kind == "f":
        xs = [raw(np.nan_to_num(x)) for x in xs]          # NaN and signed-zero ties are RCCL's own
        for x in xs:
            x[x == 0] = 0.0
    exp = [raw(x.copy()) for x in xs]
    assert oracle.allreduce(op, dt, xs, exp) == 0
    sb, rb = todev(xs[rank]), dzeros(xs[rank].nbytes)
    rc = L.MPI_Allreduce(sb.data_ptr(), rb.data_ptr(), count, dt, op, C.MPI_COMM_WORLD)
    if rc: fails.append(f"allreduce {opn} {dtn} rc={rc} {msx.last_error()}")
    else: check(f"allreduce {opn} {dtn}", fromdev(rb, xs[rank]), exp[rank], xs if tol else None)
    ip = todev(xs[rank])
    rc = L.MPI_Allreduce(IN_PLACE, ip.data_ptr(), count, dt, op, C.MPI_COMM_WORLD)
    if rc: fails.append(f"allreduce in place {opn} {dtn} rc={rc} {msx.last_error()}")
    else: check(f"allreduce in place {opn} {dtn}", fromdev(ip, xs[rank]), exp[rank], xs if tol else None)
    # host operands keep the reference-order plane (all ranks agree on it)
    hb = raw(np.zeros_like(xs[rank]))
    rc = L.MPI_Allreduce(xs[rank].ctypes.data, hb.ctypes.data, count, dt, op, C.MPI_COMM_WORLD)
    if rc: fails.append(f"allreduce host {opn} {dtn} rc={rc} {msx.last_error()}")
    else: check(f"allreduce host {opn} {dtn}", hb, exp[rank])

# MPI_Reduce at every root, and MPI_Iallreduce through the engine worker
for root in range(p):
    rng = np.random.default_rng(200 + root)
    xs = [raw(rng.uniform(-1, 1, 70003).astype(np.float32)) for _ in range(p)]
    e = raw(np.zeros_like(xs[0]))
    assert oracle.reduce(C.MPI_SUM, C.MPI_FLOAT, root, xs, e) == 0
    sb, rb = todev(xs[rank]), dzeros(xs[rank].nbytes)
    rc = L.MPI_Reduce(sb.data_ptr(), rb.data_ptr(), 70003, C.MPI_FLOAT, C.MPI_SUM, root, C.MPI_COMM_WORLD)
    if rc: fails.append(f"reduce root={root} rc={rc} {msx.last_error()}")
    elif rank == root: check(f"reduce root={root}", fromdev(rb, xs[0]), e, xs)
xs = inputs("MPI_MAX", "MPI_INT", 1 << 18, 300)
exp = [raw(x.copy()) for x in xs]
assert oracle.allreduce(C.MPI_MAX, C.MPI_INT, xs, exp) == 0
sb, rb = todev(xs[rank]), dzeros(xs[rank].nbytes)
req = ctypes.c_int()
rc = L.MPI_Iallreduce(sb.data_ptr(), rb.data_ptr(), 1 << 18, C.MPI_INT, C.MPI_MAX, C.MPI_COMM_WORLD, ctypes.byref(req))
rc = rc or L.MPI_Wait(ctypes.byref(req), ctypes.c_void_p(1))
if rc: fails.append(f"iallreduce rc={rc} {msx.last_error()}")
else: check("iallreduce", fromdev(rb, xs[rank]), exp[rank])

# reduce_scatter: equal blocks -> ncclReduceScatter (also in place); ragged -> reference order
for i, (per, ragged) in enumerate([(40000, False), (7, False), (20000, True)]):
    counts = [per + ((k % 2) * 3 if ragged else 0) for k in range(p)]
    rng = np.random.default_rng(400 + i)
    xs = [raw(rng.uniform(-1, 1, sum(counts)).astype(np.float32)) for _ in range(p)]
    ex = [raw(np.zeros(c, xs[0].dtype)) for c in counts]
    assert oracle.reduce_scatter(C.MPI_SUM, C.MPI_FLOAT, counts, xs, ex) == 0
    off = sum(counts[:rank])
    mine = [x[off:off + counts[rank]] for x in xs]
    cnt = (ctypes.c_int * p)(*counts)
    sb, rb = todev(xs[rank]), dzeros(counts[rank] * 4)
    rc = L.MPI_Reduce_scatter(sb.data_ptr(), rb.data_ptr(), cnt, C.MPI_FLOAT, C.MPI_SUM, C.MPI_COMM_WORLD)
    if rc: fails.append(f"reduce_scatter {per} rc={rc} {msx.last_error()}")
    else: check(f"reduce_scatter {per}", fromdev(rb, ex[rank], counts[rank]), ex[rank], None if ragged else mine)
    ip = todev(xs[rank])
    rc = L.MPI_Reduce_scatter(IN_PLACE, ip.data_ptr(), cnt, C.MPI_FLOAT, C.MPI_SUM, C.MPI_COMM_WORLD)
    if rc: fails.append(f"reduce_scatter in place {per} rc={rc} {msx.last_error()}")
    else: check(f"reduce_scatter in place {per}", fromdev(ip, ex[rank], counts[rank]), ex[rank],
                None if ragged else mine)

L.msx_engine_transport.restype = ctypes.c_char_p
print("TRANSPORT", L.msx_engine_transport().decode(), flush=True)
print("RESULT", rank, p, len(fails), checked, fails[:6], flush=True)
L.MPI_Finalize()
'''


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_rccl_native_collectives_one_rank_per_gpu():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    n_dev = torch.cuda.device_count()
    if n_dev < 2:
        pytest.skip("needs >= 2 GPUs (one rank per GPU)")
    p = min(n_dev, 8)                     # every visible GPU
    port = _free_port()
    procs = []
    for r in range(p):
        env = dict(os.environ)
        env.update({"MSX_SIZE": str(p), "MSX_RANK": str(r), "MSX_DEVICE": str(r),
                    "MSX_BOOTSTRAP_PORT": str(port), "MSX_BOOTSTRAP_ADDR": "127.0.0.1",
                    "MSX_BOOTSTRAP_TIMEOUT": "180", "MSX_TRANSPORT": "rccl_native",
                    "MSX_FLAG_TIMEOUT_MS": "60000"})
        procs.append(subprocess.Popen([sys.executable, "-c", f"REPO={REPO!r}\n" + textwrap.dedent(WORKER)],
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env))
    results = []
    for pr in procs:
        try:
            o, e = pr.communicate(timeout=400)
        except subprocess.TimeoutExpired:
            pr.kill()
            o, e = pr.communicate()
        results.append((pr.returncode, o, e))
    for rc, o, e in results:
        assert rc == 0, (o + e)[-3000:]
        line = [l for l in o.splitlines() if l.startswith("RESULT")]
        assert line, (o + e)[-3000:]
        assert line[0].split()[3] == "0", line[0]
        used = [l.split()[1] for l in o.splitlines() if l.startswith("TRANSPORT")]
        assert used == ["rccl_native"], used
