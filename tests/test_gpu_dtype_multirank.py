"""GPU: reduction collectives with a user-defined op on a DERIVED datatype,
1-3 MPI processes sharing one GPU.

Only user ops accept derived datatypes (the builtin ops' check tables reject
them, op.cpp:739-1883).  Each rank's contribution travels as the image of the
type's byte span, the user function runs on the typed layout (MPID_Uop_call),
and results are written back through the type map only (the non-contiguous
MPIR_Localcopy, mpid/pt2pt.cpp:770-948): the gaps of every receive buffer must
keep their bytes.  The op is an integer add walking the type map (commutative
and associative, so every schedule gives the same exact answer); expected
values come from the oracle's type map (oracle/msx_dtype_oracle.py).
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
import ctypes, os, sys
sys.path.insert(0, os.path.join(REPO, "microsoft-mpi_amd")); sys.path.insert(0, REPO)
import numpy as np, torch
import msx
from oracle import msx_dtype_oracle as O
C = msx.C
L = msx.init(errors_return=True)
r_, s_ = ctypes.c_int(), ctypes.c_int()
L.MPI_Comm_rank(C.MPI_COMM_WORLD, ctypes.byref(r_)); L.MPI_Comm_size(C.MPI_COMM_WORLD, ctypes.byref(s_))
rank, p = r_.value, s_.value
fails = []
def chk(tag, got, exp):
    if np.asarray(got).tobytes() != np.asarray(exp).tobytes():
        fails.append(tag)
def ok(rc, tag):
    if rc != 0:
        fails.append(f"{tag} rc={rc} {msx.last_error()}")
    return rc == 0

# vector(5, 2, 3) of MPI_INT: 2 ints every 3, extent 13 ints
t = ctypes.c_int()
assert L.MPI_Type_vector(5, 2, 3, C.MPI_INT, ctypes.byref(t)) == 0
assert L.MPI_Type_commit(ctypes.byref(t)) == 0
T = O.vector(5, 2, 3, O.predefined(C.MPI_INT))
EXT = T.extent // 4
def idx(count, base=0):
    return np.array([base + i * EXT + d // 4 for i in range(count) for d, _ in T.typemap], dtype=np.int64)

calls = []
UF = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int))
def add(invec, inoutvec, n, dt):
    calls.append((n[0], dt[0]))
    k = idx(n[0])
    size = int(k.max()) + 1
    x = np.ctypeslib.as_array((ctypes.c_int * size).from_address(invec))
    y = np.ctypeslib.as_array((ctypes.c_int * size).from_address(inoutvec))
    y[k] += x[k]
cb = UF(add)
op = ctypes.c_int()
assert L.MPI_Op_create(cb, 1, ctypes.byref(op)) == 0

COUNT = 3 * p                     # instances per call (reduce_scatter: 3 per rank)
N = COUNT * EXT + 8
contrib = lambda r: ((np.arange(N) * 7 + r * 1000) % 9973).astype(np.int32)
SENT = -7
def dev(a):
    t_ = torch.from_numpy(a.copy()).cuda()
    torch.cuda.synchronize()
    return t_
send = dev(contrib(rank))
total = sum(contrib(r).astype(np.int64) for r in range(p)).astype(np.int32)
K = idx(COUNT)

# Allreduce: mapped elements = sum over ranks, gaps keep the sentinel
recv = dev(np.full(N, SENT, np.int32))
ok(L.MPI_Allreduce(send.data_ptr(), recv.data_ptr(), COUNT, t.value, op.value, C.MPI_COMM_WORLD), "allreduce")
e = np.full(N, SENT, np.int32); e[K] = total[K]
chk("allreduce", recv.cpu().numpy(), e)
if calls and calls[-1][1] != t.value:
    fails.append("user fn got another datatype")

# Reduce at the last rank (host receive buffer there)
root = p - 1
hrecv = np.full(N, SENT, np.int32)
ok(L.MPI_Reduce(send.data_ptr(), hrecv.ctypes.data, COUNT, t.value, op.value, root, C.MPI_COMM_WORLD), "reduce")
if rank == root:
    chk("reduce", hrecv, e)

# Reduce_scatter_block: 3 instances per rank
rs = dev(np.full(3 * EXT + 8, SENT, np.int32))
ok(L.MPI_Reduce_scatter_block(send.data_ptr(), rs.data_ptr(), 3, t.value, op.value, C.MPI_COMM_WORLD), "rsb")
er = np.full(3 * EXT + 8, SENT, np.int32)
mine = idx(3, base=rank * 3 * EXT)
er[idx(3)] = total[mine]
chk("reduce_scatter_block", rs.cpu().numpy(), er)

# Scan: prefix sums over ranks 0..rank
sc = dev(np.full(N, SENT, np.int32))
ok(L.MPI_Scan(send.data_ptr(), sc.data_ptr(), COUNT, t.value, op.value, C.MPI_COMM_WORLD), "scan")
pre = sum(contrib(r).astype(np.int64) for r in range(rank + 1)).astype(np.int32)
es = np.full(N, SENT, np.int32); es[K] = pre[K]
chk("scan", sc.cpu().numpy(), es)

# Iallreduce in place
ip = dev(contrib(rank))
req = ctypes.c_int()
ok(L.MPI_Iallreduce(ctypes.c_void_p(C.MPI_IN_PLACE), ip.data_ptr(), COUNT, t.value, op.value, C.MPI_COMM_WORLD,
                    ctypes.byref(req)), "iallreduce")
ok(L.MPI_Wait(ctypes.byref(req), ctypes.c_void_p(1)), "wait")
ei = contrib(rank).copy(); ei[K] = total[K]
chk("iallreduce in place", ip.cpu().numpy(), ei)

# a builtin op still rejects the derived type (check table) -> MPI_ERR_OP
if L.MPI_Allreduce(send.data_ptr(), recv.data_ptr(), COUNT, t.value, C.MPI_SUM, C.MPI_COMM_WORLD) != C.MPI_ERR_OP:
    fails.append("builtin op accepted a derived type")
print("RESULT", rank, p, len(fails), fails[:6], flush=True)
L.MPI_Finalize()
'''


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.parametrize("p,switch", [(1, None), (2, None), (3, None), (3, "0")])
def test_user_op_collectives_on_derived_type(p, switch):
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
        if switch is not None:    # moved flat switch points (the oracle in the worker reads them too)
            for k in ("ALLREDUCE_SHORT_MSG", "REDUCE_SHORT_MSG", "REDSCAT_COMMUTATIVE_LONG_MSG"):
                env["MPICH_DEFAULT_" + k] = switch
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
