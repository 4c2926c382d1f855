"""GPU: generalized active-target synchronisation (MPI_Win_post / start /
complete / wait / test), 2-4 MPI processes sharing one GPU.

Reference: api/mpi_win.cpp:1331-1381, 1487-1537, 1566-1613, 1769-1808
(validation) and mpid/win.cpp:3689-4088 (MPID_Win_post / start / complete /
wait): an origin's operations reach a target only after the target posted,
and the target's MPI_Win_wait returns only after every origin of the posted
group completed, with the operations applied.  Here complete ships each
queued operation to the target's service thread, which applies it with the op
kernels on the target's GPU before the completion count is raised.  Expected
values are closed forms over integer data (exact).
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
import numpy as np, torch
import msx
C = msx.C
L = msx.init(errors_return=True)
r_, s_ = ctypes.c_int(), ctypes.c_int()
L.MPI_Comm_rank(C.MPI_COMM_WORLD, ctypes.byref(r_)); L.MPI_Comm_size(C.MPI_COMM_WORLD, ctypes.byref(s_))
rank, p = r_.value, s_.value
HOSTWIN = os.environ.get("HOSTWIN") == "1"
fails = []
def ok(rc, tag):
    if rc != 0:
        fails.append(f"{tag} rc={rc} {msx.last_error()}")
    return rc == 0
def cls(rc):
    c = ctypes.c_int(); L.MPI_Error_class(rc, ctypes.byref(c)); return c.value

N = 4 << 20                                   # int32 elements per window (16 MiB)
if HOSTWIN:
    hw = np.zeros(N, np.int32); base = hw.ctypes.data
    read = lambda: hw.copy()
else:
    dw = torch.zeros(N, dtype=torch.int32, device="cuda"); torch.cuda.synchronize(); base = dw.data_ptr()
    read = lambda: (torch.cuda.synchronize(), dw.cpu().numpy())[1]
win = ctypes.c_int()
ok(L.MPI_Win_create(ctypes.c_void_p(base), N * 4, 4, C.MPI_INFO_NULL, C.MPI_COMM_WORLD, ctypes.byref(win)), "create")
W = win.value
wg = ctypes.c_int()
ok(L.MPI_Comm_group(C.MPI_COMM_WORLD, ctypes.byref(wg)), "comm_group")
def group(ranks):
    g = ctypes.c_int()
    a = (ctypes.c_int * max(len(ranks), 1))(*ranks)
    ok(L.MPI_Group_incl(wg.value, len(ranks), a, ctypes.byref(g)), "incl")
    return g
nxt, prv = (rank + 1) % p, (rank - 1) % p
M = 65536

# 1. ring: expose to the previous rank, access the next one; a put into
#    [0, M) and an accumulate into [M, 2M) of the next rank's window
gp, gn = group([prv]), group([nxt])
for it in range(3):
    ok(L.MPI_Win_post(gp.value, 0, W), "post ring")
    ok(L.MPI_Win_start(gn.value, 0, W), "start ring")
    src = (np.arange(M, dtype=np.int32) + 1000 * rank + it)
    ok(L.MPI_Put(src.ctypes.data, M, C.MPI_INT, nxt, 0, M, C.MPI_INT, W), "put ring")
    ok(L.MPI_Accumulate(src.ctypes.data, M, C.MPI_INT, nxt, M, M, C.MPI_INT, C.MPI_SUM, W), "acc ring")
    ok(L.MPI_Win_complete(W), "complete ring")
    ok(L.MPI_Win_wait(W), "wait ring")
    # after wait the previous rank's operations of this epoch are in my window
    w = read()
    if not np.array_equal(w[:M], np.arange(M, dtype=np.int32) + 1000 * prv + it):
        fails.append(f"ring put epoch {it}")
    exp_acc = sum(np.arange(M, dtype=np.int64) + 1000 * prv + j for j in range(it + 1)).astype(np.int32)
    if not np.array_equal(w[M:2 * M], exp_acc):
        fails.append(f"ring accumulate epoch {it}")

# 2. everybody with everybody (self included): accumulate a rank-specific
#    vector into every window's region [2M, 3M); MPI_Win_test polls the exposure
ok(L.MPI_Win_post(wg.value, C.MPI_MODE_NOSTORE, W), "post all")
ok(L.MPI_Win_start(wg.value, 0, W), "start all")
v = np.arange(M, dtype=np.int32) * (rank + 1)
for t in range(p):
    ok(L.MPI_Accumulate(v.ctypes.data, M, C.MPI_INT, t, 2 * M, M, C.MPI_INT, C.MPI_SUM, W), "acc all")
ok(L.MPI_Win_complete(W), "complete all")
flag, polls = ctypes.c_int(0), 0
t_end = time.time() + 120
while not flag.value and time.time() < t_end:
    ok(L.MPI_Win_test(W, ctypes.byref(flag)), "test all")
    polls += 1
if not flag.value:
    fails.append("MPI_Win_test never completed")
w = read()
if not np.array_equal(w[2 * M:3 * M], np.arange(M, dtype=np.int32) * (p * (p + 1) // 2)):
    fails.append("all-to-all accumulate")

# 3. a subset: rank 0 exposes to everybody else, who fetch the ring data of
#    rank 0's window back with MPI_Get; rank 0's own access group is empty
others = group(list(range(1, p)))
z = group([0])
got = np.zeros(M, np.int32)
if rank == 0:
    ok(L.MPI_Win_post(others.value, C.MPI_MODE_NOPUT, W), "post subset")
    ok(L.MPI_Win_start(C.MPI_GROUP_EMPTY, 0, W), "start empty")
    ok(L.MPI_Win_complete(W), "complete empty")
    ok(L.MPI_Win_wait(W), "wait subset")
else:
    ok(L.MPI_Win_start(z.value, 0, W), "start subset")
    ok(L.MPI_Get(got.ctypes.data, M, C.MPI_INT, 0, 0, M, C.MPI_INT, W), "get subset")
    ok(L.MPI_Win_complete(W), "complete subset")
    # rank 0's [0, M) holds the put of rank p-1, epoch 2
    if not np.array_equal(got, np.arange(M, dtype=np.int32) + 1000 * (p - 1) + 2):
        fails.append("get in an access epoch")

# 4. MPI_MODE_NOCHECK: the post is known to precede the start (a barrier
#    orders them), so complete does not wait for it
if rank == 0:
    ok(L.MPI_Win_post(others.value, 0, W), "post nocheck")
L.MPI_Barrier(C.MPI_COMM_WORLD)
if rank != 0:
    ok(L.MPI_Win_start(z.value, C.MPI_MODE_NOCHECK, W), "start nocheck")
    one = np.full(16, rank, np.int32)
    ok(L.MPI_Put(one.ctypes.data, 16, C.MPI_INT, 0, 3 * M + 16 * rank, 16, C.MPI_INT, W), "put nocheck")
    ok(L.MPI_Win_complete(W), "complete nocheck")
else:
    ok(L.MPI_Win_wait(W), "wait nocheck")
    w = read()
    for o in range(1, p):
        if not np.all(w[3 * M + 16 * o: 3 * M + 16 * (o + 1)] == o):
            fails.append(f"nocheck put of {o}")

# 5. a large transfer within one epoch (pieces larger than a staging slot)
BIG = (8 << 20) // 4
ok(L.MPI_Win_post(gp.value, 0, W), "post big")
ok(L.MPI_Win_start(gn.value, 0, W), "start big")
big = (np.arange(BIG, dtype=np.int64) * 7 + rank).astype(np.int32)
ok(L.MPI_Put(big.ctypes.data, BIG, C.MPI_INT, nxt, N - BIG, BIG, C.MPI_INT, W), "put big")
ok(L.MPI_Win_complete(W), "complete big")
ok(L.MPI_Win_wait(W), "wait big")
if not np.array_equal(read()[N - BIG:], (np.arange(BIG, dtype=np.int64) * 7 + prv).astype(np.int32)):
    fails.append("big put")

# 6. errors: a group member outside the window's communicator, epoch rules
sub = ctypes.c_int()
ok(L.MPI_Comm_split(C.MPI_COMM_WORLD, rank, 0, ctypes.byref(sub)), "split")
sw = ctypes.c_int()
ok(L.MPI_Win_create(ctypes.c_void_p(base), 64, 4, C.MPI_INFO_NULL, sub.value, ctypes.byref(sw)), "create sub")
L.MPI_Win_set_errhandler(sw.value, C.MPI_ERRORS_RETURN)
if p > 1 and cls(L.MPI_Win_post(wg.value, 0, sw.value)) != C.MPI_ERR_GROUP:
    fails.append("post with a foreign group")
if cls(L.MPI_Win_complete(sw.value)) != C.MPI_ERR_RMA_SYNC:
    fails.append("complete without start")
ok(L.MPI_Win_free(ctypes.byref(sw)), "free sub")
ok(L.MPI_Comm_free(ctypes.byref(sub)), "comm free")
for g in (gp, gn, others, z, wg):
    L.MPI_Group_free(ctypes.byref(g))
ok(L.MPI_Win_free(ctypes.byref(win)), "free")
print("RESULT", rank, p, len(fails), fails[:6], flush=True)
L.MPI_Finalize()
'''


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.parametrize("p,hostwin", [(1, False), (2, False), (3, False), (4, False), (3, True)])
def test_post_start_complete_wait(p, hostwin):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    port = _free_port()
    procs = []
    for r in range(p):
        env = dict(os.environ)
        env.update({"MSX_SIZE": str(p), "MSX_RANK": str(r), "MSX_DEVICE": "0",
                    "MSX_BOOTSTRAP_PORT": str(port), "MSX_BOOTSTRAP_ADDR": "127.0.0.1",
                    "MSX_BOOTSTRAP_TIMEOUT": "180", "HOSTWIN": "1" if hostwin else "0",
                    "MSX_RMA_BYTES": "16777216"})   # 16 MiB RMA area: section 5 spans several staging slots
        procs.append(subprocess.Popen([sys.executable, "-c", f"REPO={REPO!r}\n" + textwrap.dedent(WORKER)],
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env))
    results = []
    for pr in procs:
        try:
            o, e = pr.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            pr.kill()
            o, e = pr.communicate()
        results.append((pr.returncode, o, e))
    for rc, o, e in results:
        assert rc == 0, (o + e)[-3000:]
        line = [l for l in o.splitlines() if l.startswith("RESULT")]
        assert line, (o + e)[-3000:]
        assert line[0].split()[3] == "0", line[0]
