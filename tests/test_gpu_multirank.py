"""GPU: the multi-rank collectives end to end, several MPI processes per GPU.

One MI355X box has one GPU, so p = 2, 3, 4 ranks share it: the engine's IPC
peer mapping, bootstrap hub, schedule-faithful combine kernels and allgather
copies all run for real (peer HBM is the same HBM here).  Each rank derives
every rank's input from a shared seed and compares its result with the
oracle's step-by-step simulation of the reference schedule, bit for bit.
"""
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
import ctypes, os, sys, time
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
fails = []

def raw(a):
    return np.frombuffer(bytearray(a.tobytes()), dtype=a.dtype)

def dzeros(*a, **k):
    t = torch.zeros(*a, **k)
    torch.cuda.synchronize()      # the library's streams do not order after torch's
    return t

# the harness's own transfers: page-locked by default (tests/_xfer.py, DESIGN.md §2)
from _xfer import todev, fromdev, pinned_dev, SENT_DEV, SENT_HOST

def where_wrong(tag, got, exp, dev_res, dev_in=None, own=None):
    # Which copy holds the wrong bytes (DESIGN.md §2): the device result
    # compared on the GPU with an independent upload of the expected bytes;
    # host elements still holding the readback sentinel (never written by the
    # device-to-host copy); the rank's own send buffer on the GPU against its
    # input (an upload that lost bytes).  Reported, never retried.
    ne = exp.size * exp.dtype.itemsize
    bad = np.nonzero(got != exp)[0]
    sent = np.frombuffer(np.full(exp.dtype.itemsize, SENT_HOST, np.uint8).tobytes(), exp.dtype)[0]
    unwritten = int(np.count_nonzero(got[bad] == sent))
    d = dev_res[:ne].view(torch.uint8) != pinned_dev(exp)
    dbad = torch.nonzero(d.view(-1, exp.dtype.itemsize).any(1)).flatten().cpu().numpy()
    msg = (f"{tag}: host {bad.size} wrong ({unwritten} hold the readback sentinel); "
           f"device result {dbad.size} wrong" + (f" [{dbad[0]}..{dbad[-1]}]" if dbad.size else ""))
    if dev_in is not None:
        u = dev_in[:own.nbytes].view(torch.uint8) != pinned_dev(own)
        ubad = torch.nonzero(u.view(-1, own.dtype.itemsize).any(1)).flatten().cpu().numpy()
        sd = int((dev_in[:own.nbytes][u] == SENT_DEV).sum().item())
        msg += f"; own send buffer {ubad.size} wrong" + (
            f" [{ubad[0]}..{ubad[-1]}, {sd} bytes sentinel]" if ubad.size else "")
    again = fromdev(dev_res, exp)
    return msg + f"; second readback {'clean' if again.tobytes() == exp.tobytes() else 'same error'}"

def check(tag, got, exp):
    if got.tobytes() != exp.tobytes():
        # where it differs (element ranges), for diagnosing a mismatch from one run
        g, e = np.frombuffer(got.tobytes(), np.uint8), np.frombuffer(exp.tobytes(), np.uint8)
        if g.size == e.size and exp.itemsize:
            bad = np.nonzero(g.reshape(-1, exp.itemsize) != e.reshape(-1, exp.itemsize))[0]
            bad = np.unique(bad)
            tag = f"{tag} [{bad.size} differ, first {bad[0]} last {bad[-1]}]" if bad.size else tag
        fails.append(tag)

def inputs(op, dt, count, seed):
    rng = np.random.default_rng(seed)
    return [raw(gen(KIND[dt], op, count, rng)) for _ in range(p)]

ALLREDUCE = [("MPI_SUM", "MPI_FLOAT", 1000), ("MPI_SUM", "MPI_FLOAT", 100003),
             ("MPI_MAX", "MPI_FLOAT", 70001), ("MPI_MAX", "MPI_DOUBLE", 50),
             ("MPI_BAND", "MPI_UINT64_T", 65536), ("MPI_SUM", "MPI_INT8_T", 300001),
             ("MPI_MAXLOC", "MPI_DOUBLE_INT", 40000), ("MPI_PROD", "MPI_C_FLOAT_COMPLEX", 33333),
             ("MPI_LXOR", "MPI_C_BOOL", 777)]
for i, (opn, dtn, count) in enumerate(ALLREDUCE):
    op, dt = getattr(C, opn), getattr(C, dtn)
    xs = inputs(opn, dtn, count, 1000 + i)
    exp = [raw(x.copy()) for x in xs]
    assert oracle.allreduce(op, dt, xs, exp) == 0
    for mode in ("dev", "inplace", "host"):
        if mode == "dev":
            sb, rb = todev(xs[rank]), dzeros(xs[rank].nbytes, dtype=torch.uint8, device="cuda")
            rc = L.MPI_Allreduce(sb.data_ptr(), rb.data_ptr(), count, dt, op, C.MPI_COMM_WORLD)
            got = fromdev(rb, xs[rank])
        elif mode == "inplace":
            rb = todev(xs[rank])
            rc = L.MPI_Allreduce(ctypes.c_void_p(-1 & 0xffffffffffffffff), rb.data_ptr(), count, dt, op,
                                 C.MPI_COMM_WORLD)
            got = fromdev(rb, xs[rank])
        else:
            hb = raw(np.zeros_like(xs[rank]))
            rc = L.MPI_Allreduce(xs[rank].ctypes.data, hb.ctypes.data, count, dt, op, C.MPI_COMM_WORLD)
            got = hb
        if rc != 0:
            fails.append(f"allreduce {opn} {dtn} {count} {mode} rc={rc} {msx.last_error()}")
            continue
        check(f"allreduce {opn} {dtn} {count} {mode}", got, exp[rank])

RS = [("MPI_MAX", "MPI_DOUBLE", 1000), ("MPI_SUM", "MPI_FLOAT", 40000), ("MPI_SUM", "MPI_FLOAT", 7),
      ("MPI_BXOR", "MPI_INT", 20000)]
for i, (opn, dtn, per) in enumerate(RS):
    op, dt = getattr(C, opn), getattr(C, dtn)
    counts = [per + (k % 2) * 3 for k in range(p)]
    tot = sum(counts)
    xs = inputs(opn, dtn, tot, 2000 + i)
    exp = [raw(np.zeros(c, dtype=xs[0].dtype)) for c in counts]
    assert oracle.reduce_scatter(op, dt, counts, xs, exp) == 0
    cnt = (ctypes.c_int * p)(*counts)
    for mode in ("dev", "inplace"):
        if mode == "dev":
            sb = todev(xs[rank])
            rb = dzeros(max(counts[rank] * xs[0].dtype.itemsize, 1), dtype=torch.uint8, device="cuda")
            rc = L.MPI_Reduce_scatter(sb.data_ptr(), rb.data_ptr(), cnt, dt, op, C.MPI_COMM_WORLD)
        else:
            rb = todev(xs[rank])
            rc = L.MPI_Reduce_scatter(ctypes.c_void_p(-1 & 0xffffffffffffffff), rb.data_ptr(), cnt, dt, op,
                                      C.MPI_COMM_WORLD)
        if rc != 0:
            fails.append(f"reduce_scatter {opn} {dtn} {per} {mode} rc={rc} {msx.last_error()}")
            continue
        check(f"reduce_scatter {opn} {dtn} {per} {mode}", fromdev(rb, exp[rank], counts[rank]), exp[rank])

# MPI_Reduce, binomial (small) and Rabenseifner (> 64 KiB) orders, several roots
for i, (opn, dtn, count) in enumerate([("MPI_SUM", "MPI_FLOAT", 5000), ("MPI_SUM", "MPI_FLOAT", 70003),
                                       ("MPI_MAX", "MPI_DOUBLE", 3000), ("MPI_MAX", "MPI_DOUBLE", 40000)]):
    op, dt = getattr(C, opn), getattr(C, dtn)
    xs = inputs(opn, dtn, count, 3000 + i)
    for root in sorted({0, p - 1, p // 2}):
        exp = raw(np.zeros_like(xs[0]))
        assert oracle.reduce(op, dt, root, xs, exp) == 0
        sb = todev(xs[rank])
        rb = dzeros(xs[rank].nbytes, dtype=torch.uint8, device="cuda")
        rc = L.MPI_Reduce(sb.data_ptr(), rb.data_ptr(), count, dt, op, root, C.MPI_COMM_WORLD)
        if rc != 0:
            fails.append(f"reduce {opn} {count} root={root} rc={rc} {msx.last_error()}")
        elif rank == root:
            check(f"reduce {opn} {dtn} {count} root={root}", fromdev(rb, xs[rank]), exp)

# MPI_Scan / MPI_Exscan (recursive-doubling task lists of the reference)
for i, (opn, dtn, count) in enumerate([("MPI_SUM", "MPI_FLOAT", 20001), ("MPI_MAX", "MPI_FLOAT", 3000),
                                       ("MPI_PROD", "MPI_DOUBLE_COMPLEX", 1000)]):
    op, dt = getattr(C, opn), getattr(C, dtn)
    xs = inputs(opn, dtn, count, 5000 + i)
    for excl in (False, True):
        exp = [raw(np.zeros_like(xs[0])) for _ in range(p)]
        assert oracle.scan(op, dt, xs, exp, exclusive=excl) == 0
        sb = todev(xs[rank])
        rb = dzeros(xs[rank].nbytes, dtype=torch.uint8, device="cuda")
        fn = L.MPI_Exscan if excl else L.MPI_Scan
        fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        rc = fn(sb.data_ptr(), rb.data_ptr(), count, dt, op, C.MPI_COMM_WORLD)
        if rc != 0:
            fails.append(f"scan {opn} excl={excl} rc={rc} {msx.last_error()}")
        elif not (excl and rank == 0):
            check(f"scan {opn} {dtn} excl={excl}", fromdev(rb, xs[rank]), exp[rank])
        # MPI_Iscan / MPI_Iexscan: same task order, completed in MPI_Wait
        rb2 = dzeros(xs[rank].nbytes, dtype=torch.uint8, device="cuda")
        req = ctypes.c_int()
        fi = L.MPI_Iexscan if excl else L.MPI_Iscan
        rc = fi(ctypes.c_void_p(sb.data_ptr()), ctypes.c_void_p(rb2.data_ptr()), count, dt, op, C.MPI_COMM_WORLD,
                ctypes.byref(req))
        if rc == 0:
            rc = L.MPI_Wait(ctypes.byref(req), ctypes.c_void_p(1))
        if rc != 0:
            fails.append(f"iscan {opn} excl={excl} rc={rc} {msx.last_error()}")
        elif not (excl and rank == 0):
            check(f"iscan {opn} {dtn} excl={excl}", fromdev(rb2, xs[rank]), exp[rank])
        # MPI_IN_PLACE: the input is read from recvbuf, the result replaces it
        rb3 = todev(xs[rank])
        rc = fn(ctypes.c_void_p(-1), rb3.data_ptr(), count, dt, op, C.MPI_COMM_WORLD)
        if rc != 0:
            fails.append(f"scan in place {opn} excl={excl} rc={rc} {msx.last_error()}")
        elif not (excl and rank == 0):
            check(f"scan in place {opn} {dtn} excl={excl}", fromdev(rb3, xs[rank]), exp[rank])
        # small pageable host buffers (below the pin threshold): staged for the kernels
        hs, hr = raw(xs[rank]), raw(np.zeros_like(xs[rank]))
        rc = fn(hs.ctypes.data, hr.ctypes.data, count, dt, op, C.MPI_COMM_WORLD)
        if rc != 0:
            fails.append(f"scan host {opn} excl={excl} rc={rc} {msx.last_error()}")
        elif not (excl and rank == 0):
            check(f"scan host {opn} {dtn} excl={excl}", hr, exp[rank])

# Host (pageable) buffers of 1 MiB and more: pinned for the call and used
# in place by the kernels (allreduce send/recv and in place, reduce_scatter,
# reduce at the last rank, scan), checked against the reference schedules
cnt = (3 << 20) // 4 + 5
xs = inputs("MPI_SUM", "MPI_FLOAT", cnt, 7000)
exp = [raw(x.copy()) for x in xs]
assert oracle.allreduce(C.MPI_SUM, C.MPI_FLOAT, xs, exp) == 0
hb = raw(np.zeros_like(xs[rank]))
rc = L.MPI_Allreduce(xs[rank].ctypes.data, hb.ctypes.data, cnt, C.MPI_FLOAT, C.MPI_SUM, C.MPI_COMM_WORLD)
if rc: fails.append(f"host allreduce rc={rc} {msx.last_error()}")
else: check("host allreduce pinned", hb, exp[rank])
hi = raw(xs[rank].copy())
rc = L.MPI_Allreduce(ctypes.c_void_p(-1 & 0xffffffffffffffff), hi.ctypes.data, cnt, C.MPI_FLOAT, C.MPI_SUM,
                     C.MPI_COMM_WORLD)
if rc: fails.append(f"host allreduce in place rc={rc} {msx.last_error()}")
else: check("host allreduce in place pinned", hi, exp[rank])
er = raw(np.zeros_like(xs[0]))
assert oracle.reduce(C.MPI_SUM, C.MPI_FLOAT, p - 1, xs, er) == 0
hr = raw(np.zeros_like(xs[rank]))
rc = L.MPI_Reduce(xs[rank].ctypes.data, hr.ctypes.data, cnt, C.MPI_FLOAT, C.MPI_SUM, p - 1, C.MPI_COMM_WORLD)
if rc: fails.append(f"host reduce rc={rc} {msx.last_error()}")
elif rank == p - 1: check("host reduce pinned", hr, er)
counts_h = [(1 << 20) // 8 + 3 * k for k in range(p)]
xh = inputs("MPI_MAX", "MPI_DOUBLE", sum(counts_h), 7001)
eh = [raw(np.zeros(c, xh[0].dtype)) for c in counts_h]
assert oracle.reduce_scatter(C.MPI_MAX, C.MPI_DOUBLE, counts_h, xh, eh) == 0
ch = (ctypes.c_int * p)(*counts_h)
rh = raw(np.zeros(counts_h[rank], xh[0].dtype))
rc = L.MPI_Reduce_scatter(xh[rank].ctypes.data, rh.ctypes.data, ch, C.MPI_DOUBLE, C.MPI_MAX, C.MPI_COMM_WORLD)
if rc: fails.append(f"host reduce_scatter rc={rc} {msx.last_error()}")
else: check("host reduce_scatter pinned", rh, eh[rank])
ih = raw(xh[rank].copy())
rc = L.MPI_Reduce_scatter(ctypes.c_void_p(-1 & 0xffffffffffffffff), ih.ctypes.data, ch, C.MPI_DOUBLE, C.MPI_MAX,
                          C.MPI_COMM_WORLD)
if rc: fails.append(f"host reduce_scatter in place rc={rc} {msx.last_error()}")
else: check("host reduce_scatter in place pinned", ih[:counts_h[rank]], eh[rank])
es = [raw(np.zeros_like(xs[0])) for _ in range(p)]
assert oracle.scan(C.MPI_SUM, C.MPI_FLOAT, xs, es, exclusive=False) == 0
hs = raw(np.zeros_like(xs[rank]))
L.MPI_Scan.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]
rc = L.MPI_Scan(xs[rank].ctypes.data, hs.ctypes.data, cnt, C.MPI_FLOAT, C.MPI_SUM, C.MPI_COMM_WORLD)
if rc: fails.append(f"host scan rc={rc} {msx.last_error()}")
else: check("host scan pinned", hs, es[rank])

# MPI_Ireduce / MPI_Ireduce_scatter_block / MPI_Ireduce_scatter in flight together,
# completed by one MPI_Waitall (issue order = execution order on every rank)
cnt = 30001
xr = inputs("MPI_SUM", "MPI_FLOAT", cnt, 6000)
er = raw(np.zeros_like(xr[0]))
assert oracle.ireduce(C.MPI_SUM, C.MPI_FLOAT, p - 1, xr, er) == 0      # NBC task list: root-relative ranks
per = 5003
xs_b = inputs("MPI_MAX", "MPI_DOUBLE", per * p, 6001)
es_b = [raw(np.zeros(per, xs_b[0].dtype)) for _ in range(p)]
assert oracle.reduce_scatter(C.MPI_MAX, C.MPI_DOUBLE, [per] * p, xs_b, es_b) == 0
counts_v = [1000 + 7 * k for k in range(p)]
xs_v = inputs("MPI_BXOR", "MPI_INT", sum(counts_v), 6002)
es_v = [raw(np.zeros(c, xs_v[0].dtype)) for c in counts_v]
assert oracle.reduce_scatter(C.MPI_BXOR, C.MPI_INT, counts_v, xs_v, es_v) == 0
d_r, o_r = todev(xr[rank]), dzeros(xr[rank].nbytes, dtype=torch.uint8, device="cuda")
d_b, o_b = todev(xs_b[rank]), dzeros(per * 8, dtype=torch.uint8, device="cuda")
d_v, o_v = todev(xs_v[rank]), dzeros(counts_v[rank] * 4, dtype=torch.uint8, device="cuda")
reqs = (ctypes.c_int * 3)()
cv = (ctypes.c_int * p)(*counts_v)
rcs = [L.MPI_Ireduce(d_r.data_ptr(), o_r.data_ptr(), cnt, C.MPI_FLOAT, C.MPI_SUM, p - 1, C.MPI_COMM_WORLD,
                     ctypes.cast(ctypes.addressof(reqs) + 0, ctypes.POINTER(ctypes.c_int))),
       L.MPI_Ireduce_scatter_block(d_b.data_ptr(), o_b.data_ptr(), per, C.MPI_DOUBLE, C.MPI_MAX, C.MPI_COMM_WORLD,
                                   ctypes.cast(ctypes.addressof(reqs) + 4, ctypes.POINTER(ctypes.c_int))),
       L.MPI_Ireduce_scatter(d_v.data_ptr(), o_v.data_ptr(), cv, C.MPI_INT, C.MPI_BXOR, C.MPI_COMM_WORLD,
                             ctypes.cast(ctypes.addressof(reqs) + 8, ctypes.POINTER(ctypes.c_int)))]
if any(rcs):
    fails.append(f"nbc start rc={rcs} {msx.last_error()}")
else:
    rc = L.MPI_Waitall(3, reqs, ctypes.c_void_p(1))
    if rc:
        fails.append(f"waitall rc={rc} {msx.last_error()}")
    else:
        if rank == p - 1:
            check("ireduce", fromdev(o_r, xr[rank]), er)
        check("ireduce_scatter_block", fromdev(o_b, es_b[rank]), es_b[rank])
        check("ireduce_scatter", fromdev(o_v, es_v[rank]), es_v[rank])
        if list(reqs) != [C.MPI_REQUEST_NULL] * 3:
            fails.append(f"waitall left requests {list(reqs)}")

# MPI_Iallreduce BAND u64 (config 5 op/type) overlapped with host compute
xs = inputs("MPI_BAND", "MPI_UINT64_T", 1 << 18, 4000)
exp = [raw(x.copy()) for x in xs]
oracle.allreduce(C.MPI_BAND, C.MPI_UINT64_T, xs, exp)
sb, rb = todev(xs[rank]), dzeros(xs[rank].nbytes, dtype=torch.uint8, device="cuda")
req = ctypes.c_int()
rc = L.MPI_Iallreduce(sb.data_ptr(), rb.data_ptr(), 1 << 18, C.MPI_UINT64_T, C.MPI_BAND, C.MPI_COMM_WORLD,
                      ctypes.byref(req))
host = np.random.default_rng(1).random(1 << 20)
flag, polls = ctypes.c_int(0), 0
while rc == 0 and not flag.value:
    host = 1.0001 * host + 0.5           # host work between tests
    rc = L.MPI_Test(ctypes.byref(req), ctypes.byref(flag), ctypes.c_void_p(1))
    polls += 1
if rc != 0:
    fails.append(f"iallreduce rc={rc} {msx.last_error()}")
else:
    check("iallreduce band u64", fromdev(rb, xs[rank]), exp[rank])
assert req.value == C.MPI_REQUEST_NULL

# Two nonblocking allreduces in flight, completed by MPI_Waitany (one per call,
# indices in issue order) and a Testsome/Testall poll (api/mpi_completion.cpp)
xa = inputs("MPI_SUM", "MPI_INT", 200003, 4100)
xb = inputs("MPI_MAX", "MPI_DOUBLE", 77777, 4101)
ea, eb = [raw(x.copy()) for x in xa], [raw(x.copy()) for x in xb]
oracle.allreduce(C.MPI_SUM, C.MPI_INT, xa, ea)
oracle.allreduce(C.MPI_MAX, C.MPI_DOUBLE, xb, eb)
sa, ra = todev(xa[rank]), dzeros(xa[rank].nbytes, dtype=torch.uint8, device="cuda")
sb2, rb2 = todev(xb[rank]), dzeros(xb[rank].nbytes, dtype=torch.uint8, device="cuda")
reqs = (ctypes.c_int * 2)()
rcs = [L.MPI_Iallreduce(sa.data_ptr(), ra.data_ptr(), 200003, C.MPI_INT, C.MPI_SUM, C.MPI_COMM_WORLD,
                        ctypes.cast(ctypes.addressof(reqs), ctypes.POINTER(ctypes.c_int))),
       L.MPI_Iallreduce(sb2.data_ptr(), rb2.data_ptr(), 77777, C.MPI_DOUBLE, C.MPI_MAX, C.MPI_COMM_WORLD,
                        ctypes.cast(ctypes.addressof(reqs) + 4, ctypes.POINTER(ctypes.c_int)))]
seen = []
if any(rcs):
    fails.append(f"waitany start rc={rcs} {msx.last_error()}")
else:
    idx = ctypes.c_int(-1)
    for _ in range(2):
        rc = L.MPI_Waitany(2, reqs, ctypes.byref(idx), ctypes.c_void_p(1))
        if rc: fails.append(f"waitany rc={rc} {msx.last_error()}")
        seen.append(idx.value)
    rc = L.MPI_Waitany(2, reqs, ctypes.byref(idx), ctypes.c_void_p(1))
    if rc or idx.value != -32766 or sorted(seen) != [0, 1]:
        fails.append(f"waitany order {seen} last={idx.value} rc={rc}")
    check("waitany allreduce int", fromdev(ra, xa[rank]), ea[rank])
    check("waitany allreduce dbl", fromdev(rb2, xb[rank]), eb[rank])
rc = L.MPI_Iallreduce(sa.data_ptr(), ra.data_ptr(), 200003, C.MPI_INT, C.MPI_SUM, C.MPI_COMM_WORLD,
                      ctypes.cast(ctypes.addressof(reqs), ctypes.POINTER(ctypes.c_int)))
flag, polls = ctypes.c_int(0), 0
while rc == 0 and not flag.value:
    rc = L.MPI_Testall(1, reqs, ctypes.byref(flag), ctypes.c_void_p(1))
    polls += 1
if rc: fails.append(f"testall rc={rc} {msx.last_error()}")
else: check("testall allreduce int", fromdev(ra, xa[rank]), ea[rank])

# Back-to-back stress of the barrier-free allreduce paths (GPU arrival flags,
# alternating IN / OUT halves; above MSX_TWO_STEP_MAX the host-barrier schedules)
# interleaved with the other window users: small rooted reduces (the same
# arrival-flag path, non-roots push to the root only), a chunked large
# allreduce (full barrier first), non-blocking calls through the engine
# worker, in-place calls.
from _stress import ivec, stress_n, classify

def stress_diag(it, n, got, tot):
    # which mechanism explains the wrong elements (tests/_stress.py, DESIGN.md §2)
    bad = np.nonzero(got != tot)[0]
    hyp = classify(it, n, bad, got[bad], tot[bad], p, rank)
    sample = ", ".join(f"{int(k)}:{int(a)}/{int(b)}" for k, a, b in zip(bad[:3], got[bad[:3]], tot[bad[:3]]))
    return (f"[{bad.size} differ, first {bad[0]} last {bad[-1]}; got/exp {sample}; "
            f"explained by: {', '.join(hyp[:8]) or 'none of the tested'}]")

passes = int(os.environ.get("MSX_STRESS_PASSES", "1"))
for it in range(240 * passes):
    # recursive doubling / binomial (GPU flags) up to 64 Ki ints, the two-step
    # Rabenseifner (GPU flags) or, above MSX_TWO_STEP_MAX, the host-barrier one
    n = stress_n(it)
    if passes > 1 and it % 240 == 0:
        print("PASS", it // 240, len(fails), flush=True)
    tot = sum(ivec(it, r, n).astype(np.int64) for r in range(p)).astype(np.int32)
    sb = todev(ivec(it, rank, n))
    if it % 7 == 3:                        # rooted reduce: arrival flags, push to the root only
        root = it % p
        rb = dzeros(n * 4, dtype=torch.uint8, device="cuda")
        rc = L.MPI_Reduce(sb.data_ptr(), rb.data_ptr(), n, C.MPI_INT, C.MPI_SUM, root, C.MPI_COMM_WORLD)
        if rc:
            fails.append(f"stress reduce {it} rc={rc}")
        elif rank == root:
            check(f"stress reduce {it}", fromdev(rb, tot), tot)
        continue
    if it % 9 == 4:                        # reduce_scatter_block: one-step (GPU flags) or host barriers
        full = [ivec(it, r, n * p) for r in range(p)]
        mine_tot = sum(f[rank * n:(rank + 1) * n].astype(np.int64) for f in full).astype(np.int32)
        sb = todev(full[rank])
        rb = dzeros(n * 4, dtype=torch.uint8, device="cuda")
        rc = L.MPI_Reduce_scatter_block(sb.data_ptr(), rb.data_ptr(), n, C.MPI_INT, C.MPI_SUM, C.MPI_COMM_WORLD)
        if rc:
            fails.append(f"stress rsb {it} rc={rc} {msx.last_error()}")
            break
        got_rs = fromdev(rb, mine_tot)
        check(f"stress rsb {it} n={n}", got_rs, mine_tot)
        if got_rs.tobytes() != mine_tot.tobytes():
            fails.append(where_wrong(f"stress rsb {it}", got_rs, mine_tot, rb, sb, full[rank]))
        continue
    if it % 11 == 5:                       # non-blocking, through the worker
        rb = dzeros(n * 4, dtype=torch.uint8, device="cuda")
        req = ctypes.c_int()
        rc = L.MPI_Iallreduce(sb.data_ptr(), rb.data_ptr(), n, C.MPI_INT, C.MPI_SUM, C.MPI_COMM_WORLD,
                              ctypes.byref(req))
        rc = rc or L.MPI_Wait(ctypes.byref(req), ctypes.c_void_p(1))
    elif it % 5 == 2:                      # in place
        rb = sb
        rc = L.MPI_Allreduce(ctypes.c_void_p(C.MPI_IN_PLACE), rb.data_ptr(), n, C.MPI_INT, C.MPI_SUM,
                             C.MPI_COMM_WORLD)
    else:
        rb = dzeros(n * 4, dtype=torch.uint8, device="cuda")
        rc = L.MPI_Allreduce(sb.data_ptr(), rb.data_ptr(), n, C.MPI_INT, C.MPI_SUM, C.MPI_COMM_WORLD)
    if rc:
        fails.append(f"stress allreduce {it} rc={rc} {msx.last_error()}")
        break
    got = fromdev(rb, tot)
    if got.tobytes() != tot.tobytes():
        fails.append(f"stress allreduce {it} n={n} {stress_diag(it, n, got, tot)}")
        inplace = rb is sb
        fails.append(where_wrong(f"stress allreduce {it}", got, tot, rb, None if inplace else sb,
                                 None if inplace else ivec(it, rank, n)))

L.msx_engine_transport.restype = ctypes.c_char_p
print("TRANSPORT", L.msx_engine_transport().decode(), flush=True)
st = (ctypes.c_double * 8)()
L.msx_engine_stats(st, 8, 0)
print("FLAGCALLS", int(st[7]), flush=True)       # GPU-flag Rabenseifner calls of this rank
print("RESULT", rank, p, len(fails), fails[:16], flush=True)
L.MPI_Finalize()
'''


def _assert_all_ranks(results):
    """Every rank exited 0 and reported no failure; on failure the message holds
    EVERY rank's RESULT line (or its output tail), not just the first one, so a
    single run tells whether the peers saw the same wrong bytes."""
    lines, ok = [], True
    for r, (rc, o, e) in enumerate(results):
        res = [l for l in o.splitlines() if l.startswith("RESULT")]
        if rc != 0 or not res:
            ok = False
            lines.append(f"rank {r}: rc={rc} {(o + e)[-1500:]}")
        else:
            ok = ok and res[0].split()[3] == "0"
            lines.append(res[0])
    assert ok, "\n".join(lines)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


# Every case runs all p ranks on ONE GPU (the GPU box has one): same-HBM IPC,
# so these pin the schedules and the flag/barrier protocol, not cross-GPU
# (xGMI) memory ordering -- that needs the driver's multi-GPU node.
@pytest.mark.parametrize("p,chunk,transport,rd_flags", [(2, None, None, None), (3, 65536, None, None),
                                                        (4, 1 << 20, None, None), (5, None, None, None),
                                                        (3, 65536, "rccl", None), (8, None, None, None),
                                                        (7, 1 << 20, None, None), (8, None, None, "pageable"),
                                                        (4, None, None, "ts512k"), (6, None, None, None),
                                                        (4, None, None, "switch0"),
                                                        (3, None, None, "switch0"), (5, None, None, "switchmax"),
                                                        (5, 65536, None, "switch0"), (7, None, None, "switchmax"),
                                                        (8, None, None, "switch0"), (3, None, None, "staged"),
                                                        (3, None, "rccl_native", None),
                                                        (2, None, None, "+ts"), (5, None, None, "+ts"),
                                                        (8, None, None, "+ts"), (3, 65536, None, "+ts"),
                                                        (4, 65536, None, "+ts"), (8, None, None, "switch0+ts")])
def test_collectives_p_ranks_on_one_gpu(p, chunk, transport, rd_flags):
    """`+ts`: the GPU-flag Rabenseifner schedules (two-step allreduce / reduce,
    one-step reduce_scatter, flag scan) forced on.  Ranks that share a GPU
    default to the host-barrier schedules since round 4, so the
    flag schedules the one-rank-per-GPU deployment runs are tested here by
    asking for them."""
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
        mode = rd_flags
        if mode and mode.endswith("+ts"):
            env["MSX_TWO_STEP_MAX"] = str(1 << 62)
            mode = mode[:-3] or None
        if chunk:
            env["MSX_CHUNK_BYTES"] = str(chunk)     # many chunks, pieces across block edges
        if transport:
            env["MSX_TRANSPORT"] = transport
        if mode == "pageable":
            # the harness's own transfers pageable (tests/_xfer.py) with
            # sentinels: a hole in a pageable copy is then located by
            # where_wrong instead of hidden by page-locked transfers
            env["MSX_TEST_PINNED"] = "0"
        elif mode in ("switch0", "switchmax"):
            # the reference's flat switch points moved (mpid/env.cpp:514-608): at 0
            # every allreduce of >= pof2 elements is Rabenseifner (blocks of a few
            # elements) and every reduce_scatter pairwise; the oracle simulation
            # in the worker reads the same variables
            v = "0" if mode == "switch0" else "2147483647"
            for k in ("ALLREDUCE_SHORT_MSG", "REDUCE_SHORT_MSG", "REDSCAT_COMMUTATIVE_LONG_MSG"):
                env["MPICH_DEFAULT_" + k] = v
        elif mode == "staged":
            # host buffers staged through HBM: no call-scoped pinning, no bounce buffers
            env["MSX_TEST_HOST_PIN_MIN"] = str(1 << 40)
            env["MSX_TEST_HOST_BOUNCE_MAX"] = "0"
        elif mode == "ts512k":
            env["MSX_TWO_STEP_MAX"] = str(512 << 10)   # two-step and host-barrier Rabenseifner alternate
        elif mode is not None:
            raise AssertionError(f"unknown mode {mode}")
        procs.append(subprocess.Popen([sys.executable, "-c", f"REPO={REPO!r}\n" + textwrap.dedent(WORKER)],
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env))
    results = []
    for pr in procs:
        try:
            o, e = pr.communicate(timeout=400 * int(os.environ.get("MSX_STRESS_PASSES", "1")))
        except subprocess.TimeoutExpired:
            pr.kill()
            o, e = pr.communicate()
        results.append((pr.returncode, o, e))
    _assert_all_ranks(results)
    for rc, o, e in results:
        used = [l.split()[1] for l in o.splitlines() if l.startswith("TRANSPORT")]
        # RCCL needs one GPU per rank: these ranks all run on GPU 0 (MSX_DEVICE=0,
        # whatever the node has), so they keep the IPC engine
        assert used == ["ipc"], used
        # ranks sharing the GPU run the GPU-flag Rabenseifner schedules only
        # when asked: the stress loop's 100,003- and
        # 300,001-int calls take them with `+ts` / `ts512k`, never by default
        flag_calls = [int(l.split()[1]) for l in o.splitlines() if l.startswith("FLAGCALLS")]
        if transport is None and "MSX_TWO_STEP_MAX" not in os.environ:   # (a run may force it for all)
            if rd_flags and (rd_flags.endswith("+ts") or rd_flags == "ts512k"):
                assert flag_calls and flag_calls[0] > 0, (rd_flags, flag_calls)
            else:
                assert flag_calls == [0], (rd_flags, flag_calls)


# One rank per GPU -- the deployment the north star names.  The one-GPU box
# skips these; on a node with >= 2 visible GPUs they execute the cross-GPU data
# paths that the shared-GPU cases above cannot: IPC windows opened on another
# device (xGMI remote writes, system-scope write-through, peer flag polls) and
# the RCCL send/recv plane, each checked bit for bit against the oracle.
@pytest.mark.parametrize("sched", ["default", "host_barrier", "pipeline"])
@pytest.mark.parametrize("transport", ["ipc", "rccl"])
def test_collectives_one_rank_per_gpu(transport, sched):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    n_dev = torch.cuda.device_count()
    if n_dev < 2:
        pytest.skip("needs >= 2 GPUs (one rank per GPU)")
    p = min(n_dev, 8)                     # every visible GPU, as the 8-GPU configs
    port = _free_port()
    procs = []
    for r in range(p):
        env = dict(os.environ)
        env.update({"MSX_SIZE": str(p), "MSX_RANK": str(r), "MSX_DEVICE": str(r),
                    "MSX_BOOTSTRAP_PORT": str(port), "MSX_BOOTSTRAP_ADDR": "127.0.0.1",
                    "MSX_BOOTSTRAP_TIMEOUT": "180", "MSX_TRANSPORT": transport,
                    "MSX_FLAG_TIMEOUT_MS": "60000"})
        if sched == "host_barrier":
            env["MSX_TWO_STEP_MAX"] = "0"       # the host-barrier Rabenseifner schedules only
        elif sched == "pipeline":
            env["MSX_TWO_STEP_MAX"] = str(1 << 62)   # the opt-in GPU-flag pipeline at every size
        procs.append(subprocess.Popen([sys.executable, "-c", f"REPO={REPO!r}\n" + textwrap.dedent(WORKER)],
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env))
    results = []
    for pr in procs:
        try:
            o, e = pr.communicate(timeout=400 * int(os.environ.get("MSX_STRESS_PASSES", "1")))
        except subprocess.TimeoutExpired:
            pr.kill()
            o, e = pr.communicate()
        results.append((pr.returncode, o, e))
    _assert_all_ranks(results)
    for rc, o, e in results:
        used = [l.split()[1] for l in o.splitlines() if l.startswith("TRANSPORT")]
        assert used == [transport], used
