"""GPU: remote one-sided operations through TWO-LEVEL compact target types.

A derived target datatype travels to the target with the operation as its
serialized layout (the reference ships the dataloop); 3-D subarrays and
vectors of strided vectors now travel in the two-level compact form
(first, len, stride, n, stride2, n2) instead of an explicit run list.  Two
ranks on one GPU: every rank accumulates (fence epoch) into a 3-D fp32
subarray of the next rank's window, puts through an hvector-of-vector type
into a second window, and reads a subarray back with MPI_Get; each target
checks its window bit for bit against numpy slicing (fp32 SUM: one add per
element in (origin rank, issue) order, so exact).
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
C = msx.C
L = msx.init(errors_return=True)
r_, s_ = ctypes.c_int(), ctypes.c_int()
L.MPI_Comm_rank(C.MPI_COMM_WORLD, ctypes.byref(r_)); L.MPI_Comm_size(C.MPI_COMM_WORLD, ctypes.byref(s_))
rank, p = r_.value, s_.value
fails = []
def ok(rc, tag):
    if rc != 0:
        fails.append(f"{tag} rc={rc} {msx.last_error()}")
ia = lambda v: (ctypes.c_int * len(v))(*v)
def new(fn, *a):
    t = ctypes.c_int()
    assert fn(*a, ctypes.byref(t)) == 0, msx.last_error()
    assert L.MPI_Type_commit(ctypes.byref(t)) == 0
    return t

dims, sub, st = (12, 20, 36), (5, 7, 11), (4, 9, 13)
T3 = new(L.MPI_Type_create_subarray, 3, ia(dims), ia(sub), ia(st), C.MPI_ORDER_C, C.MPI_FLOAT)
inner = new(L.MPI_Type_vector, 9, 1, 3, C.MPI_INT)                      # every 3rd int of 27
VV = new(L.MPI_Type_create_hvector, 6, 1, 40 * 4, inner.value)           # 6 rows of 40 ints
base = lambda r: (np.arange(np.prod(dims)) % 997 + 1000 * r).astype(np.float32).reshape(dims)
contrib = lambda r: ((np.arange(np.prod(sub)) % 13) * 0.25 + r + 1).astype(np.float32)
w3 = torch.from_numpy(base(rank).reshape(-1)).cuda()
wi = torch.zeros(6 * 40, dtype=torch.int32, device="cuda")
src = torch.from_numpy(contrib(rank)).cuda()
isrc = torch.arange(54, dtype=torch.int32, device="cuda") + 100 * rank
back = torch.zeros(int(np.prod(sub)), device="cuda")
torch.cuda.synchronize()
W3, WI = ctypes.c_int(), ctypes.c_int()
assert L.MPI_Win_create(w3.data_ptr(), w3.numel() * 4, 4, C.MPI_INFO_NULL, C.MPI_COMM_WORLD, ctypes.byref(W3)) == 0
assert L.MPI_Win_create(wi.data_ptr(), wi.numel() * 4, 4, C.MPI_INFO_NULL, C.MPI_COMM_WORLD, ctypes.byref(WI)) == 0
for w in (W3, WI):
    ok(L.MPI_Win_fence(0, w), "open fence")
nxt, prv = (rank + 1) % p, (rank - 1) % p
n_sub = int(np.prod(sub))
ok(L.MPI_Accumulate(src.data_ptr(), n_sub, C.MPI_FLOAT, nxt, 0, 1, T3.value, C.MPI_SUM, W3), "acc 3d")
ok(L.MPI_Put(isrc.data_ptr(), 54, C.MPI_INT, nxt, 0, 1, VV.value, WI), "put vv")
for w in (W3, WI):
    ok(L.MPI_Win_fence(0, w), "fence")
ok(L.MPI_Get(back.data_ptr(), n_sub, C.MPI_FLOAT, nxt, 0, 1, T3.value, W3), "get 3d")
ok(L.MPI_Win_fence(0, W3), "fence get")
torch.cuda.synchronize()
e3 = base(rank).copy()
blk = e3[st[0]:st[0] + sub[0], st[1]:st[1] + sub[1], st[2]:st[2] + sub[2]]
blk += contrib(prv).reshape(sub)                       # the one origin writing into my window
if w3.cpu().numpy().tobytes() != e3.reshape(-1).tobytes():
    fails.append("3-D subarray accumulate")
ei = np.zeros((6, 40), np.int32)
ei[:, 0:27:3] = (np.arange(54, dtype=np.int32) + 100 * prv).reshape(6, 9)
if wi.cpu().numpy().tobytes() != ei.reshape(-1).tobytes():
    fails.append("hvector-of-vector put")
en = base(nxt).copy()
en[st[0]:st[0] + sub[0], st[1]:st[1] + sub[1], st[2]:st[2] + sub[2]] += contrib(rank).reshape(sub)
eb = en[st[0]:st[0] + sub[0], st[1]:st[1] + sub[1], st[2]:st[2] + sub[2]].reshape(-1)
if back.cpu().numpy().tobytes() != eb.tobytes():
    fails.append("3-D subarray get")
for w in (W3, WI):
    ok(L.MPI_Win_free(ctypes.byref(w)), "free")
print("RESULT", rank, p, len(fails), fails[:6], flush=True)
L.MPI_Finalize()
'''


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.parametrize("p,compact2", [(2, "1"), (3, "1"), (2, "0")])
def test_rma_two_level_compact_target_types(p, compact2):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    port = _free_port()
    procs = []
    for r in range(p):
        env = dict(os.environ)
        env.update({"MSX_SIZE": str(p), "MSX_RANK": str(r), "MSX_DEVICE": "0",
                    "MSX_BOOTSTRAP_PORT": str(port), "MSX_BOOTSTRAP_ADDR": "127.0.0.1",
                    "MSX_BOOTSTRAP_TIMEOUT": "180",
                    "MSX_TEST_DT_COMPACT2": compact2})      # 0: the explicit run-list form, for contrast
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
