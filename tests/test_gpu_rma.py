"""GPU: one-sided accumulate (MPI_Win + fence), several MPI processes per GPU.

Every rank exposes device windows (and one host-memory window); each rank
issues Put / Get / Accumulate / Get_accumulate / Fetch_and_op /
Compare_and_swap against its peers and itself, closes the epoch with
MPI_Win_fence and checks every window and every fetched value bit for bit.

Application order (reference: mpid/win.cpp:1537-1610, packethandling.cpp
:2917-3060): an operation whose target is the calling rank is applied at the
call (MPIDI_Win_local_accumulate); remote operations are applied by the target
at the fence.  The reference applies remote operations in arrival order; here
they are applied in (origin rank, issue) order, so the expected values below
follow that order: the target's own operations first, then origins ascending.
Expected floating-point values come from oracle.reduce_local applied in that
order.
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
import msx, oracle
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

W, K = 4096, 1000
BIG = int(os.environ.get("RMA_BIG", "50000"))
init_i = lambda r: (np.arange(W, dtype=np.int64) * 3 + r * 1000).astype(np.int32)
wi_t = torch.from_numpy(init_i(rank)).cuda()
rng = lambda r: np.random.default_rng(100 + r)
init_f = lambda r: (rng(r).standard_normal(BIG) * 10.0 ** rng(r).integers(-3, 4, BIG)).astype(np.float32)
wf_t = torch.from_numpy(init_f(rank)).cuda()
wh = np.full(256, float(rank), np.float64)            # host-memory window
torch.cuda.synchronize()
wi, wf, whw = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
assert L.MPI_Win_create(wi_t.data_ptr(), W * 4, 4, C.MPI_INFO_NULL, C.MPI_COMM_WORLD, ctypes.byref(wi)) == 0
assert L.MPI_Win_create(wf_t.data_ptr(), BIG * 4, 4, C.MPI_INFO_NULL, C.MPI_COMM_WORLD, ctypes.byref(wf)) == 0
assert L.MPI_Win_create(wh.ctypes.data, wh.nbytes, 8, C.MPI_INFO_NULL, C.MPI_COMM_WORLD, ctypes.byref(whw)) == 0
for w in (wi, wf, whw):
    L.MPI_Win_set_errhandler(w, C.MPI_ERRORS_RETURN)
    ok(L.MPI_Win_fence(0, w), "open fence")

I, F, D = C.MPI_INT, C.MPI_FLOAT, C.MPI_DOUBLE
contrib = lambda r: (np.arange(K) * (r + 1) - 7).astype(np.int32)
put_data = lambda r: (np.arange(K) + r * 7).astype(np.int32)
gacc_data = lambda r: ((np.arange(K) * (r + 5)) % 97).astype(np.int32)
facc = lambda r: (rng(50 + r).standard_normal(BIG)).astype(np.float32)

# device origin buffers, host result buffers (mixed placement on purpose)
c_dev = torch.from_numpy(contrib(rank)).cuda()
p_dev = torch.from_numpy(put_data(rank)).cuda()
g_dev = torch.from_numpy(gacc_data(rank)).cuda()
g_res = np.zeros(K, np.int32)
f_dev = torch.from_numpy(facc(rank)).cuda()
one = np.ones(1, np.int32); fo_res = np.zeros(1, np.int32)
cas_org = np.array([100 + rank], np.int32); cas_cmp = np.array([init_i(0)[W - 2]], np.int32)
cas_res = np.zeros(1, np.int32)
get_res = torch.zeros(K, dtype=torch.int32, device="cuda")
h_org = np.full(16, 0.5 * (rank + 1))
torch.cuda.synchronize()
last = p - 1
ok(L.MPI_Accumulate(c_dev.data_ptr(), K, I, 0, 0, K, I, C.MPI_SUM, wi), "acc")
ok(L.MPI_Put(p_dev.data_ptr(), K, I, (rank + 1) % p, K, K, I, wi), "put")
ok(L.MPI_Fetch_and_op(one.ctypes.data, fo_res.ctypes.data, I, 0, W - 1, C.MPI_SUM, wi), "fop")
ok(L.MPI_Compare_and_swap(cas_org.ctypes.data, cas_cmp.ctypes.data, cas_res.ctypes.data, I, 0, W - 2, wi), "cas")
ok(L.MPI_Get_accumulate(g_dev.data_ptr(), K, I, g_res.ctypes.data, K, I, last, 2 * K, K, I, C.MPI_MAX, wi), "gacc")
ok(L.MPI_Accumulate(f_dev.data_ptr(), BIG, F, 0, 0, BIG, F, C.MPI_SUM, wf), "facc")
ok(L.MPI_Accumulate(h_org.ctypes.data, 16, D, last, 8, 16, D, C.MPI_PROD, whw), "hacc")
for w in (wi, wf, whw):
    ok(L.MPI_Win_fence(0, w), "fence")
# a Get after the epoch that wrote it
ok(L.MPI_Get(get_res.data_ptr(), K, I, (rank + 1) % p, K, K, I, wi), "get")
ok(L.MPI_Win_fence(0, wi), "fence2")

order = lambda t: [t] + [o for o in range(p) if o != t]       # self first, then ascending
wi_h = wi_t.cpu().numpy()
if rank == 0:
    exp = init_i(0)[:K].copy()
    for o in range(p):
        exp += contrib(o)
    chk("acc int sum", wi_h[:K], exp)
    chk("fetch_and_op final", wi_h[W - 1:W], init_i(0)[W - 1:W] + p)
    chk("cas final", wi_h[W - 2:W - 1], np.array([100], np.int32))
    e = init_f(0).copy()
    for o in order(0):
        oracle.reduce_local(C.MPI_SUM, C.MPI_FLOAT, facc(o), e)
    chk("acc float sum order", wf_t.cpu().numpy(), e)
chk("put", wi_h[K:2 * K], put_data((rank - 1) % p))
chk("get", get_res.cpu().numpy(), put_data(rank))
pos = order(0).index(rank)
chk("fetch_and_op value", fo_res, init_i(0)[W - 1:W] + pos)
chk("cas value", cas_res, init_i(0)[W - 2:W - 1] if rank == 0 else np.array([100], np.int32))
cur = init_i(last)[2 * K:3 * K].copy()
for o in order(last):
    if o == rank:
        chk("gacc fetched", g_res, cur)
    cur = np.maximum(cur, gacc_data(o))
if rank == last:
    chk("gacc final", wi_h[2 * K:3 * K], cur)
    eh = np.full(256, float(last))
    for o in order(last):
        eh[8:24] *= 0.5 * (o + 1)
    chk("host window prod", wh, eh)

# out-of-bounds target: MPI_ERR_REQUEST at the fence on the origin, no effect
if p > 1:
    bad = ctypes.c_int(0)
    x = np.ones(8, np.int32)
    rc1 = L.MPI_Put(x.ctypes.data, 8, I, (rank + 1) % p, W - 4, 8, I, wi)
    rc2 = L.MPI_Win_fence(0, wi)
    if rc1 != 0 or rc2 != C.MPI_ERR_REQUEST:
        fails.append(f"oob rc={rc1},{rc2}")
    chk("oob no effect", wi_t.cpu().numpy()[W - 4:W - 2], wi_h[W - 4:W - 2])
for w in (wi, wf, whw):
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


@pytest.mark.parametrize("p,chunk", [(1, None), (2, None), (3, 65536), (4, 1 << 20)])
def test_rma_fence_epochs_on_one_gpu(p, chunk):
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
        if chunk:
            env["MSX_CHUNK_BYTES"] = str(chunk)     # several fence rounds, split operations
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
