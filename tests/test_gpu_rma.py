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


# ---- derived datatypes in one-sided operations --------------------------------
# Origin types are packed on the origin's GPU, target types travel as their
# flattened layout and are walked by the gfx950 unpack / accumulate / pack
# kernels at the target (the reference ships the dataloop and walks it in
# do_accumulate_op, packethandling.cpp:2969-3004).  Expected values: the
# oracle's type maps (oracle/msx_dtype_oracle.py) applied with numpy.
WORKER_DT = r'''
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
def new(fn, *a):
    t = ctypes.c_int()
    assert fn(*a, ctypes.byref(t)) == 0, msx.last_error()
    assert L.MPI_Type_commit(ctypes.byref(t)) == 0
    return t.value
ia = lambda v, ct=ctypes.c_int: (ct * len(v))(*v)
D, I = C.MPI_DOUBLE, C.MPI_INT
N = 64
# a column of an N x N row-major fp64 matrix, resized so consecutive columns follow
col0 = new(L.MPI_Type_vector, N, 1, N, D)
col = new(L.MPI_Type_create_resized, col0, 0, 8)
ocol = O.resized(O.vector(N, 1, N, O.predefined(D)), 0, 8)
# a 4 x 8 block at (10, 20) of the matrix
blk = new(L.MPI_Type_create_subarray, 2, ia([N, N]), ia([4, 8]), ia([10, 20]), C.MPI_ORDER_C, D)
oblk = O.subarray([N, N], [4, 8], [10, 20], True, O.predefined(D))
# origin side: every other element of a 64-vector
ev = new(L.MPI_Type_vector, 32, 1, 2, D)
oev = O.vector(32, 1, 2, O.predefined(D))
# irregular int blocks for BXOR
ix = new(L.MPI_Type_indexed, 3, ia([5, 1, 9]), ia([0, 11, 30]), I)
oix = O.indexed([5, 1, 9], [0, 11, 30], O.predefined(I))
idx = lambda t, esz, count=1, base=0: np.array([base + i * t.extent // esz + d // esz
                                              for i in range(count) for d, _ in t.typemap])

init_m = lambda r: (np.arange(N * N) % 1000 + 10000 * r).astype(np.float64)
wm_t = torch.from_numpy(init_m(rank)).cuda()
init_x = lambda r: ((np.arange(256) * 2654435761 + r) % (1 << 31)).astype(np.int32)
wx_t = torch.from_numpy(init_x(rank)).cuda()
wh = np.arange(512, dtype=np.float64) - 100.0 * rank        # host (pageable) window
torch.cuda.synchronize()
wm, wx, whw = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
assert L.MPI_Win_create(wm_t.data_ptr(), N * N * 8, 8, C.MPI_INFO_NULL, C.MPI_COMM_WORLD, ctypes.byref(wm)) == 0
assert L.MPI_Win_create(wx_t.data_ptr(), 256 * 4, 4, C.MPI_INFO_NULL, C.MPI_COMM_WORLD, ctypes.byref(wx)) == 0
assert L.MPI_Win_create(wh.ctypes.data, wh.nbytes, 8, C.MPI_INFO_NULL, C.MPI_COMM_WORLD, ctypes.byref(whw)) == 0
for w in (wm, wx, whw):
    L.MPI_Win_set_errhandler(w, C.MPI_ERRORS_RETURN)
    ok(L.MPI_Win_fence(0, w), "open fence")

colv = lambda r: (np.arange(N) * (r + 1) + 0.5).astype(np.float64)
c_dev = torch.from_numpy(colv(rank)).cuda()
put64 = lambda r: (np.arange(64) * 3.0 + 1000 * r).astype(np.float64)
p_host = put64(rank)                                    # host origin, derived origin type
xo = lambda r: ((np.arange(15) + 1) * (0x01010101 * (r + 3))).astype(np.int32)
x_dev = torch.from_numpy(xo(rank)).cuda()
g_res = torch.zeros(64, dtype=torch.float64, device="cuda")
ga = lambda r: (np.arange(N) % 7 * 1.0 + r).astype(np.float64)
ga_host = ga(rank)
ga_res = np.zeros(N, np.float64)
torch.cuda.synchronize()
nxt, last = (rank + 1) % p, p - 1
# column `rank` of rank 0's matrix += my column (derived target, predefined origin)
ok(L.MPI_Accumulate(c_dev.data_ptr(), N, D, 0, rank, 1, col, C.MPI_SUM, wm), "acc col")
# the next rank's 4x8 block <- every other element of my 64-vector (derived both sides)
ok(L.MPI_Put(p_host.ctypes.data, 1, ev, nxt, 0, 1, blk, wm), "put blk")
# BXOR through an irregular int layout at the last rank, displaced by 40 ints
ok(L.MPI_Accumulate(x_dev.data_ptr(), 15, I, last, 40, 1, ix, C.MPI_BXOR, wx), "acc bxor")
# host window at rank 0: MAX through a column layout (stride 8 doubles, 64 rows)
ok(L.MPI_Get_accumulate(ga_host.ctypes.data, N, D, ga_res.ctypes.data, N, D, 0, 0, 1,
                        new(L.MPI_Type_vector, N, 1, 8, D), C.MPI_MAX, whw), "gacc host")
for w in (wm, wx, whw):
    ok(L.MPI_Win_fence(0, w), "fence")
# Get with a derived origin (result) type from the block written above
ok(L.MPI_Get(g_res.data_ptr(), 1, ev, nxt, 0, 1, blk, wm), "get blk")
ok(L.MPI_Win_fence(0, wm), "fence2")

order = lambda t: [t] + [o for o in range(p) if o != t]
wm_h = wm_t.cpu().numpy()
if rank == 0:
    e = init_m(0).copy()
    for o in range(p):
        e[idx(ocol, 8, base=o)] += colv(o)
    prev = (0 - 1) % p
    e[idx(oblk, 8)] = put64(prev)[idx(oev, 8)]
    chk("acc col + put blk @0", wm_h, e)
else:
    e = init_m(rank).copy()
    e[idx(oblk, 8)] = put64(rank - 1)[idx(oev, 8)]
    chk("put blk", wm_h, e)
exp_g = np.zeros(64)
exp_g[idx(oev, 8)] = put64(rank)[idx(oev, 8)]
chk("get derived result", g_res.cpu().numpy(), exp_g)
if rank == last:
    e = init_x(last).copy()
    for o in order(last):
        e[40 + idx(oix, 4)] ^= xo(o)
    chk("bxor indexed", wx_t.cpu().numpy(), e)
cur = (np.arange(512, dtype=np.float64))[::8][:N].copy()
for o in order(0):
    if o == rank:
        chk("gacc fetched", ga_res, cur)
    cur = np.maximum(cur, ga(o))
if rank == 0:
    e = np.arange(512, dtype=np.float64)
    e[0:8 * N:8] = cur
    chk("gacc host window", wh, e)
for w in (wm, wx, whw):
    ok(L.MPI_Win_free(ctypes.byref(w)), "free")
print("RESULT", rank, p, len(fails), fails[:6], flush=True)
L.MPI_Finalize()
'''


@pytest.mark.parametrize("p,chunk", [(1, None), (2, None), (3, 4096)])
def test_rma_derived_datatypes_on_one_gpu(p, chunk):
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
            env["MSX_CHUNK_BYTES"] = str(chunk)     # pieces of a derived op land in different rounds
        procs.append(subprocess.Popen([sys.executable, "-c", f"REPO={REPO!r}\n" + textwrap.dedent(WORKER_DT)],
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
