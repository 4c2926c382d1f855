"""GPU: reductions on derived communicators (MPI_Comm_split / MPI_Comm_dup /
MPI_Comm_create),
4 and 5 ranks sharing one GPU.  Each group runs the engine on its own
transport (hub, shared-memory barrier, IPC windows, arrival flags), so
collectives on WORLD and on the groups interleave freely.  Integer data:
exact closed forms in group-rank order."""
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
C = msx.C
L = msx.init(errors_return=True)
r_, s_ = ctypes.c_int(), ctypes.c_int()
L.MPI_Comm_rank(C.MPI_COMM_WORLD, ctypes.byref(r_)); L.MPI_Comm_size(C.MPI_COMM_WORLD, ctypes.byref(s_))
rank, p = r_.value, s_.value
fails = []
def ok(rc, tag):
    if rc:
        fails.append(f"{tag} rc={rc} {msx.last_error()}")
    return rc == 0
def dev(a):
    t = torch.from_numpy(np.ascontiguousarray(a)).cuda(); torch.cuda.synchronize(); return t
def host(t):
    torch.cuda.synchronize(); return t.cpu().numpy()

sub = ctypes.c_int()
ok(L.MPI_Comm_split(C.MPI_COMM_WORLD, rank % 2, rank, ctypes.byref(sub)), "split")
S = sub.value
sr, ss = ctypes.c_int(), ctypes.c_int()
L.MPI_Comm_rank(S, ctypes.byref(sr)); L.MPI_Comm_size(S, ctypes.byref(ss))
members = [r for r in range(p) if r % 2 == rank % 2]          # group order = world order
assert members[sr.value] == rank and ss.value == len(members)
dup = ctypes.c_int()
ok(L.MPI_Comm_dup(C.MPI_COMM_WORLD, ctypes.byref(dup)), "dup")

for it, n in enumerate((1, 1000, 1 << 16, 3 << 20)):       # flag path .. Rabenseifner
    x = lambda r: ((np.arange(n, dtype=np.int64) * 7 + r * 131 + it) % 65521).astype(np.int32)
    send = dev(x(rank)); recv = dev(np.zeros(n, np.int32))
    ok(L.MPI_Allreduce(send.data_ptr(), recv.data_ptr(), n, C.MPI_INT, C.MPI_SUM, S), f"sub allreduce {n}")
    exp = sum(x(r).astype(np.int64) for r in members).astype(np.int32)
    if not np.array_equal(host(recv), exp): fails.append(f"sub allreduce {n}")
    # a WORLD collective in between (its own windows)
    recv_w = dev(np.zeros(n, np.int32))
    ok(L.MPI_Allreduce(send.data_ptr(), recv_w.data_ptr(), n, C.MPI_INT, C.MPI_MAX, C.MPI_COMM_WORLD), f"world {n}")
    expw = np.max(np.stack([x(r) for r in range(p)]), axis=0)
    if not np.array_equal(host(recv_w), expw): fails.append(f"world allreduce {n}")
    # the duplicate of WORLD
    recv_d = dev(np.zeros(n, np.int32))
    ok(L.MPI_Allreduce(send.data_ptr(), recv_d.data_ptr(), n, C.MPI_INT, C.MPI_BXOR, dup.value), f"dup {n}")
    expd = np.bitwise_xor.reduce(np.stack([x(r) for r in range(p)]), axis=0)
    if not np.array_equal(host(recv_d), expd): fails.append(f"dup allreduce {n}")

# rooted reduce at group rank last, reduce_scatter_block, iallreduce on the group
g = len(members)
n = 4096 * g
x = lambda r: ((np.arange(n, dtype=np.int64) * 3 + r) % 1000).astype(np.int32)
send = dev(x(rank))
out = dev(np.zeros(n, np.int32))
ok(L.MPI_Reduce(send.data_ptr(), out.data_ptr(), n, C.MPI_INT, C.MPI_SUM, g - 1, S), "sub reduce")
tot = sum(x(r).astype(np.int64) for r in members).astype(np.int32)
if sr.value == g - 1 and not np.array_equal(host(out), tot): fails.append("sub reduce")
blk = dev(np.zeros(4096, np.int32))
ok(L.MPI_Reduce_scatter_block(send.data_ptr(), blk.data_ptr(), 4096, C.MPI_INT, C.MPI_SUM, S), "sub rsb")
if not np.array_equal(host(blk), tot[sr.value * 4096:(sr.value + 1) * 4096]): fails.append("sub rsb")
req = ctypes.c_int()
res = dev(np.zeros(n, np.int32))
ok(L.MPI_Iallreduce(send.data_ptr(), res.data_ptr(), n, C.MPI_INT, C.MPI_SUM, S, ctypes.byref(req)), "sub iallreduce")
ok(L.MPI_Wait(ctypes.byref(req), ctypes.c_void_p(1)), "wait")
if not np.array_equal(host(res), tot): fails.append("sub iallreduce")

# MPI_Comm_create from a group in reversed world order without world rank 1:
# the new ranks follow the group, so a scan accumulates in that order
wg, rg, cc = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
L.MPI_Comm_group(C.MPI_COMM_WORLD, ctypes.byref(wg))
order = [r for r in reversed(range(p)) if r != 1 or p == 1]
ok(L.MPI_Group_incl(wg.value, len(order), (ctypes.c_int * len(order))(*order), ctypes.byref(rg)), "incl")
ok(L.MPI_Comm_create(C.MPI_COMM_WORLD, rg.value, ctypes.byref(cc)), "comm_create")
if rank in order:
    k = order.index(rank)
    cr = ctypes.c_int(); L.MPI_Comm_rank(cc.value, ctypes.byref(cr))
    if cr.value != k: fails.append(f"created rank {cr.value} != {k}")
    n = 1 << 16
    x = lambda r: ((np.arange(n, dtype=np.int64) * 5 + r * 17) % 1009).astype(np.int32)
    send = dev(x(rank)); out = dev(np.zeros(n, np.int32))
    ok(L.MPI_Scan(send.data_ptr(), out.data_ptr(), n, C.MPI_INT, C.MPI_SUM, cc.value), "scan created")
    if not np.array_equal(host(out), sum(x(r).astype(np.int64) for r in order[:k + 1]).astype(np.int32)):
        fails.append("scan on the created communicator")
    ok(L.MPI_Allreduce(send.data_ptr(), out.data_ptr(), n, C.MPI_INT, C.MPI_SUM, cc.value), "allreduce created")
    if not np.array_equal(host(out), sum(x(r).astype(np.int64) for r in order).astype(np.int32)):
        fails.append("allreduce on the created communicator")
    ok(L.MPI_Comm_free(ctypes.byref(cc)), "free created")
elif cc.value != C.MPI_COMM_NULL:
    fails.append("non-member got a communicator")
L.MPI_Group_free(ctypes.byref(rg)); L.MPI_Group_free(ctypes.byref(wg))

ok(L.MPI_Comm_free(ctypes.byref(sub)), "free sub")
ok(L.MPI_Comm_free(ctypes.byref(dup)), "free dup")
print("RESULT", rank, p, len(fails), fails[:5], flush=True)
L.MPI_Finalize()
'''


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.parametrize("p", [4, 5])
def test_reductions_on_split_communicators(p):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    port = _free_port()
    procs = []
    for r in range(p):
        env = dict(os.environ)
        env.update({"MSX_SIZE": str(p), "MSX_RANK": str(r), "MSX_DEVICE": "0",
                    "MSX_BOOTSTRAP_PORT": str(port), "MSX_BOOTSTRAP_ADDR": "127.0.0.1",
                    "MSX_BOOTSTRAP_TIMEOUT": "180", "MSX_CHUNK_BYTES": str(64 << 20)})
        procs.append(subprocess.Popen([sys.executable, "-c", f"REPO={REPO!r}\n" + textwrap.dedent(WORKER)],
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env))
    for pr in procs:
        try:
            o, e = pr.communicate(timeout=300)
        except subprocess.TimeoutExpired:
            pr.kill()
            o, e = pr.communicate()
        assert pr.returncode == 0, (o + e)[-3000:]
        line = [l for l in o.splitlines() if l.startswith("RESULT")]
        assert line, (o + e)[-3000:]
        assert line[0].split()[3] == "0", line[0]
