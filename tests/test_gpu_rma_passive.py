"""GPU: passive-target one-sided communication (MPI_Win_lock / unlock /
lock_all / flush), 2-4 MPI processes sharing one GPU.

Reference: api/mpi_win.cpp:1153-1990 (validation), mpid/win.cpp:4090-4500
(lazy remote locks, blocking self lock) and the target-side apply of
packethandling.cpp:2917-3060.  Here each target's service thread applies the
requests with the op kernels on its own GPU, so the checks below also pin
atomicity: fetch-and-add under shared locks must hand out every ticket
exactly once, exclusive-lock read-modify-write cycles must not lose updates.
Expected values are closed forms over integer data (exact).
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
HOSTWIN = os.environ.get("HOSTWIN") == "1"
fails = []
def ok(rc, tag):
    if rc != 0:
        fails.append(f"{tag} rc={rc} {msx.last_error()}")
    return rc == 0
def cls(rc):
    c = ctypes.c_int(); L.MPI_Error_class(rc, ctypes.byref(c)); return c.value

N = 8 << 20                                   # int32 elements per window (32 MiB)
if HOSTWIN:
    hw = np.zeros(N, np.int32); base = hw.ctypes.data
    read = lambda: hw.copy()
else:
    dw = torch.zeros(N, dtype=torch.int32, device="cuda"); torch.cuda.synchronize(); base = dw.data_ptr()
    read = lambda: (torch.cuda.synchronize(), dw.cpu().numpy())[1]
win = ctypes.c_int()
ok(L.MPI_Win_create(ctypes.c_void_p(base), N * 4, 4, C.MPI_INFO_NULL, C.MPI_COMM_WORLD, ctypes.byref(win)), "create")
W = win.value
one = np.ones(1, np.int32)
K = 40

# 1. exclusive-lock read-modify-write (get, +1, put) on rank 0's element 0:
#    no update may be lost
for it in range(K):
    ok(L.MPI_Win_lock(C.MPI_LOCK_EXCLUSIVE, 0, 0, W), "lock excl")
    v = np.zeros(1, np.int32)
    ok(L.MPI_Get(v.ctypes.data, 1, C.MPI_INT, 0, 0, 1, C.MPI_INT, W), "get")
    ok(L.MPI_Win_flush(0, W), "flush")
    v += 1
    ok(L.MPI_Put(v.ctypes.data, 1, C.MPI_INT, 0, 0, 1, C.MPI_INT, W), "put")
    ok(L.MPI_Win_unlock(0, W), "unlock excl")

# 2. fetch-and-add tickets under shared locks (lock_all): element 1 of the last rank
last = p - 1
tickets = []
ok(L.MPI_Win_lock_all(0, W), "lock_all")
for it in range(K):
    f = np.zeros(1, np.int32)
    ok(L.MPI_Fetch_and_op(one.ctypes.data, f.ctypes.data, C.MPI_INT, last, 1, C.MPI_SUM, W), "fao")
    ok(L.MPI_Win_flush(last, W), "flush fao")
    tickets.append(int(f[0]))
# accumulate a rank-specific vector into every peer's region [1024 + 4096*r, +4096)
src = (np.arange(4096, dtype=np.int32) * (rank + 1))
for t in range(p):
    ok(L.MPI_Accumulate(src.ctypes.data, 4096, C.MPI_INT, t, 1024 + 4096 * rank, 4096, C.MPI_INT, C.MPI_SUM, W), "acc")
ok(L.MPI_Win_flush_all(W), "flush_all")
ok(L.MPI_Win_unlock_all(W), "unlock_all")

# 3. a derived target type: vector(64, 3, 7) of INT into the next rank's
#    region at 65536 + 8192*rank, then read back through the same type
T = ctypes.c_int()
L.MPI_Type_vector(64, 3, 7, C.MPI_INT, ctypes.byref(T)); L.MPI_Type_commit(ctypes.byref(T))
nxt = (rank + 1) % p
payload = (np.arange(192, dtype=np.int32) + 7000 * (rank + 1))
ok(L.MPI_Win_lock(C.MPI_LOCK_EXCLUSIVE, nxt, 0, W), "lock vec")
ok(L.MPI_Put(payload.ctypes.data, 192, C.MPI_INT, nxt, 65536 + 8192 * rank, 1, T.value, W), "put vec")
back = np.zeros(192, np.int32)
ok(L.MPI_Get(back.ctypes.data, 192, C.MPI_INT, nxt, 65536 + 8192 * rank, 1, T.value, W), "get vec")
ok(L.MPI_Win_unlock(nxt, W), "unlock vec")
if not np.array_equal(back, payload):
    fails.append("derived put/get round trip")

# 4. compare-and-swap: everybody tries to swap 0 -> 1000 + rank at element 3 of
#    rank 0; exactly one rank may win
ok(L.MPI_Win_lock(C.MPI_LOCK_SHARED, 0, 0, W), "lock cas2")
new, cmp_, res = np.array([1000 + rank], np.int32), np.array([0], np.int32), np.zeros(1, np.int32)
ok(L.MPI_Compare_and_swap(new.ctypes.data, cmp_.ctypes.data, res.ctypes.data, C.MPI_INT, 0, 3, W), "cas")
ok(L.MPI_Win_unlock(0, W), "unlock cas2")
won = np.array([1 if res[0] == 0 else 0], np.int64)

# 5. a transfer larger than one staging slot (split into pieces)
BIG = (24 << 20) // 4 if p <= 2 else (12 << 20) // 4
region = N - BIG
ok(L.MPI_Win_lock(C.MPI_LOCK_EXCLUSIVE, nxt, 0, W), "lock big")
big = (np.arange(BIG, dtype=np.int64) * 3 + rank).astype(np.int32)
if rank % 2 == 0 or p == 1:                 # even ranks write, odd ranks only read later
    ok(L.MPI_Put(big.ctypes.data, BIG, C.MPI_INT, nxt, region, BIG, C.MPI_INT, W), "put big")
ok(L.MPI_Win_unlock(nxt, W), "unlock big")

# 6. errors (reference classes): bad lock type, bad rank, double lock, unlock w/o lock
if cls(L.MPI_Win_lock(999, 0, 0, W)) != C.MPI_ERR_OTHER: fails.append("locktype")
if cls(L.MPI_Win_lock(C.MPI_LOCK_SHARED, p + 3, 0, W)) != C.MPI_ERR_RANK: fails.append("lock rank")
if cls(L.MPI_Win_unlock(nxt, W)) != C.MPI_ERR_OTHER: fails.append("unlock without lock")
ok(L.MPI_Win_lock(C.MPI_LOCK_SHARED, nxt, 0, W), "lock again 1")
if cls(L.MPI_Win_lock(C.MPI_LOCK_SHARED, nxt, 0, W)) != C.MPI_ERR_OTHER: fails.append("double lock")
ok(L.MPI_Win_unlock(nxt, W), "unlock again")
ok(L.MPI_Win_lock(C.MPI_LOCK_SHARED, C.MPI_PROC_NULL, 0, W), "lock proc_null")
ok(L.MPI_Win_unlock(C.MPI_PROC_NULL, W), "unlock proc_null")
ok(L.MPI_Win_sync(W), "sync")

L.MPI_Barrier(C.MPI_COMM_WORLD)
w = read()
if rank == 0:
    if w[0] != p * K:
        fails.append(f"lost exclusive updates: {w[0]} != {p * K}")
if rank == last:
    if w[1] != p * K:
        fails.append(f"fetch-and-add total {w[1]} != {p * K}")
for r in range(p):
    exp = np.arange(4096, dtype=np.int32) * (r + 1)
    if not np.array_equal(w[1024 + 4096 * r: 1024 + 4096 * (r + 1)], exp):
        fails.append(f"accumulate region of rank {r}")
prv = (rank - 1) % p
vt = O.vector(64, 3, 7, O.predefined(C.MPI_INT))
idx = np.array([65536 + 8192 * prv + d // 4 for d, _ in vt.typemap])
if not np.array_equal(w[idx], np.arange(192, dtype=np.int32) + 7000 * (prv + 1)):
    fails.append("derived put at target")
if rank == 0 and not (1000 <= w[3] < 1000 + p):
    fails.append(f"cas winner value {w[3]}")
if prv % 2 == 0 or p == 1:
    expb = (np.arange(BIG, dtype=np.int64) * 3 + prv).astype(np.int32)
    if not np.array_equal(w[region:], expb):
        fails.append("big put")

# tickets: all ranks together must hold 0 .. p*K-1 exactly once
tk = np.array(tickets, np.int64)
allt = np.zeros(p * K, np.int64)
wonall = np.zeros(1, np.int64)
ok(L.MPI_Allreduce(ctypes.c_void_p(won.ctypes.data), ctypes.c_void_p(wonall.ctypes.data), 1, C.MPI_INT64_T, C.MPI_SUM, C.MPI_COMM_WORLD), "won")
buf = np.zeros(p * K, np.int64); buf[rank * K:(rank + 1) * K] = tk
ok(L.MPI_Allreduce(ctypes.c_void_p(buf.ctypes.data), ctypes.c_void_p(allt.ctypes.data), p * K, C.MPI_INT64_T, C.MPI_SUM, C.MPI_COMM_WORLD), "tickets")
if sorted(allt.tolist()) != list(range(p * K)):
    fails.append("fetch-and-add tickets are not a permutation")
if wonall[0] != 1:
    fails.append(f"{wonall[0]} CAS winners")
L.MPI_Type_free(ctypes.byref(T))
ok(L.MPI_Win_free(ctypes.byref(win)), "free")

# MPI_Win_allocate: pinned host memory owned by the window; every rank adds 1
# to its own element of every window under lock_all
bp, w2 = ctypes.c_void_p(), ctypes.c_int()
ok(L.MPI_Win_allocate(4 * 64, 4, C.MPI_INFO_NULL, C.MPI_COMM_WORLD, ctypes.byref(bp), ctypes.byref(w2)), "win_allocate")
arr = np.ctypeslib.as_array((ctypes.c_int * 64).from_address(bp.value))
arr[:] = 0
L.MPI_Barrier(C.MPI_COMM_WORLD)
ok(L.MPI_Win_lock_all(0, w2.value), "lock_all 2")
for t in range(p):
    ok(L.MPI_Accumulate(one.ctypes.data, 1, C.MPI_INT, t, rank, 1, C.MPI_INT, C.MPI_SUM, w2.value), "acc 2")
ok(L.MPI_Win_unlock_all(w2.value), "unlock_all 2")
L.MPI_Barrier(C.MPI_COMM_WORLD)
if not (np.all(arr[:p] == 1) and np.all(arr[p:] == 0)):
    fails.append(f"win_allocate contents {arr[:p + 1]}")
ok(L.MPI_Win_free(ctypes.byref(w2)), "free 2")

# 7. request-based RMA (api/mpi_rma.cpp:187,486,813,1215): MPI_Rget_accumulate
#    tickets, MPI_Raccumulate (request freed), MPI_Rput / MPI_Rget round trip;
#    outside a passive-target epoch MPI_ERR_RMA_SYNC
vp, i32, i64, pr = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.POINTER(ctypes.c_int)
L.MPI_Rput.argtypes = [vp, i32, i32, i32, i64, i32, i32, i32, pr]
L.MPI_Rget.argtypes = [vp, i32, i32, i32, i64, i32, i32, i32, pr]
L.MPI_Raccumulate.argtypes = [vp, i32, i32, i32, i64, i32, i32, i32, i32, pr]
L.MPI_Rget_accumulate.argtypes = [vp, i32, i32, vp, i32, i32, i32, i64, i32, i32, i32, i32, pr]
M3 = 4096
if HOSTWIN:
    hw3 = np.zeros(M3, np.int32); b3 = hw3.ctypes.data
    read3 = lambda: hw3.copy()
else:
    dw3 = torch.zeros(M3, dtype=torch.int32, device="cuda"); torch.cuda.synchronize(); b3 = dw3.data_ptr()
    read3 = lambda: (torch.cuda.synchronize(), dw3.cpu().numpy())[1]
w3 = ctypes.c_int()
ok(L.MPI_Win_create(ctypes.c_void_p(b3), M3 * 4, 4, C.MPI_INFO_NULL, C.MPI_COMM_WORLD, ctypes.byref(w3)), "create 3")
W3 = w3.value
req = ctypes.c_int()
if cls(L.MPI_Raccumulate(one.ctypes.data, 1, C.MPI_INT, 0, 0, 1, C.MPI_INT, C.MPI_SUM, W3, ctypes.byref(req))) \
        != C.MPI_ERR_RMA_SYNC:
    fails.append("raccumulate outside an epoch")
ok(L.MPI_Win_lock_all(0, W3), "lock_all 3")
t2 = []
for it in range(10):
    f = np.zeros(1, np.int32)
    ok(L.MPI_Rget_accumulate(one.ctypes.data, 1, C.MPI_INT, f.ctypes.data, 1, C.MPI_INT, last, 0, 1, C.MPI_INT,
                             C.MPI_SUM, W3, ctypes.byref(req)), "rget_accumulate")
    ok(L.MPI_Wait(ctypes.byref(req), ctypes.c_void_p(1)), "wait rgacc")
    t2.append(int(f[0]))
vec = np.arange(256, dtype=np.int32) * (rank + 1)
for t in range(p):
    ok(L.MPI_Raccumulate(vec.ctypes.data, 256, C.MPI_INT, t, 256, 256, C.MPI_INT, C.MPI_SUM, W3, ctypes.byref(req)),
       "raccumulate")
    ok(L.MPI_Request_free(ctypes.byref(req)), "free rma request")
pv = np.arange(64, dtype=np.int32) + 100 * rank
for t in range(p):
    ok(L.MPI_Rput(pv.ctypes.data, 64, C.MPI_INT, t, 1024 + 64 * rank, 64, C.MPI_INT, W3, ctypes.byref(req)), "rput")
    ok(L.MPI_Wait(ctypes.byref(req), ctypes.c_void_p(1)), "wait rput")
bk = np.zeros(64, np.int32)
ok(L.MPI_Rget(bk.ctypes.data, 64, C.MPI_INT, nxt, 1024 + 64 * rank, 64, C.MPI_INT, W3, ctypes.byref(req)), "rget")
ok(L.MPI_Wait(ctypes.byref(req), ctypes.c_void_p(1)), "wait rget")
if not np.array_equal(bk, pv):
    fails.append("rput/rget round trip")
ok(L.MPI_Win_unlock_all(W3), "unlock_all 3")
L.MPI_Barrier(C.MPI_COMM_WORLD)
w = read3()
if rank == last and w[0] != 10 * p:
    fails.append(f"rget_accumulate total {w[0]} != {10 * p}")
if not np.array_equal(w[256:512], np.arange(256, dtype=np.int32) * sum(r + 1 for r in range(p))):
    fails.append("raccumulate region")
for r in range(p):
    if not np.array_equal(w[1024 + 64 * r:1024 + 64 * (r + 1)], np.arange(64, dtype=np.int32) + 100 * r):
        fails.append(f"rput region of rank {r}")
if len(set(t2)) != 10:
    fails.append("rget_accumulate tickets repeat")
ok(L.MPI_Win_free(ctypes.byref(w3)), "free 3")
print("RESULT", rank, p, len(fails), fails[:6], flush=True)
L.MPI_Finalize()
'''


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.parametrize("p,hostwin", [(1, False), (2, False), (3, False), (4, False), (2, True)])
def test_passive_target_rma(p, hostwin):
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
                    "MSX_RMA_BYTES": "67108864"})   # 64 MiB RMA area: section 5 spans several staging slots
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
