"""GPU: the BASELINE.json collective configs at their FULL per-rank sizes, with
the ranks sharing this box's one GPU (the 8-GPU node is the driver's):

  c3  MPI_Allreduce  MPI_SUM  MPI_FLOAT   1 GiB per rank (2 chunks of the
      default 512 MiB window), p = 2 and p = 3 (non-power-of-two fold)
  c4  MPI_Reduce_scatter_block MPI_MAX MPI_DOUBLE, 4 GiB send buffer per rank
      (536,870,912 doubles: the reference's 32-bit byte count wraps to 0 and
      selects recursive halving, reduce.cpp:1705), p = 2
  c5  MPI_Iallreduce MPI_BAND MPI_UINT64_T, 512 MiB per rank, overlapped with
      host work before MPI_Wait, p = 2
  and all three with the configs' own rank count, p = 8 (fp32 SUM checked
  against the 8-leaf balanced tree of the reference's Rabenseifner order)

Size-independent checks, computed on the GPU by every rank from the other
ranks' seeds: fp32 SUM is the reference association (x0 + x1) + x2 (IEEE adds
commute, so the fold's operand order does not change the bits), MAX over
finite doubles and BAND are exact -- all compared bit for bit."""
import os
import socket
import subprocess
import sys
import textwrap
import time

import pytest

import msx

pytestmark = pytest.mark.gpu
REPO = msx.REPO_ROOT

WORKER = r'''
import ctypes, os, sys, time
sys.path.insert(0, os.path.join(REPO, "microsoft-mpi_amd"))
import numpy as np, torch
import msx
C = msx.C
L = msx.init(errors_return=True)
r_, s_ = ctypes.c_int(), ctypes.c_int()
L.MPI_Comm_rank(C.MPI_COMM_WORLD, ctypes.byref(r_)); L.MPI_Comm_size(C.MPI_COMM_WORLD, ctypes.byref(s_))
rank, p = r_.value, s_.value
W = C.MPI_COMM_WORLD
CFG = os.environ["FULL_CFG"]
fails = []

def gen_f32(seed, n):
    g = torch.Generator(device="cuda").manual_seed(seed)
    return torch.rand(n, device="cuda", generator=g) * 2 - 1

def gen_f64(seed, n):
    g = torch.Generator(device="cuda").manual_seed(seed)
    return torch.rand(n, device="cuda", generator=g, dtype=torch.float64) * 2 - 1

def gen_u64(seed, n):
    g = torch.Generator(device="cuda").manual_seed(seed)
    # bits set with probability 1 - 2^-5 (the AND over the ranks stays non-trivial)
    x = torch.full((n,), -1, dtype=torch.int64, device="cuda")
    for _ in range(5):
        x &= torch.empty(n, dtype=torch.int64, device="cuda").random_(generator=g) | \
             torch.empty(n, dtype=torch.int64, device="cuda").random_(generator=g)
    return x

def done(tag, rc, t0):
    print(f"{tag} rc={rc} {time.perf_counter() - t0:.3f}s", file=sys.stderr, flush=True)
    if rc:
        fails.append(f"{tag} rc={rc} {msx.last_error()}")

if CFG == "c3":
    n = 1 << 28                                   # 1 GiB of fp32 per rank
    x = gen_f32(0x5EED + rank, n)
    y = torch.empty_like(x)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    done("c3 allreduce", L.MPI_Allreduce(x.data_ptr(), y.data_ptr(), n, C.MPI_FLOAT, C.MPI_SUM, W), t0)
    del x
    if p & (p - 1) == 0:
        # power of two: the balanced tree ((x0+x1)+(x2+x3))+((x4+x5)+(x6+x7)), reduce.cpp:3890-4009
        level = [gen_f32(0x5EED + r, n) for r in range(0, p, 2)]
        level = [a.add_(gen_f32(0x5EED + 2 * i + 1, n)) for i, a in enumerate(level)]
        while len(level) > 1:
            level = [level[i].add_(level[i + 1]) for i in range(0, len(level), 2)]
        exp = level[0]
    else:
        exp = gen_f32(0x5EED, n)
        for r in range(1, p):
            exp = exp + gen_f32(0x5EED + r, n)    # ((x0 + x1) + x2): the fold's tree for p = 3
    torch.cuda.synchronize()
    if not torch.equal(y.view(torch.int32), exp.view(torch.int32)):
        fails.append(f"c3: {(y != exp).sum().item()} elements differ")
elif CFG == "c4":
    n = 1 << 29                                   # 4 GiB of fp64 per rank
    per = n // p
    x = gen_f64(0xC4 + rank, n)
    y = torch.empty(per, dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    done("c4 reduce_scatter_block", L.MPI_Reduce_scatter_block(x.data_ptr(), y.data_ptr(), per, C.MPI_DOUBLE,
                                                               C.MPI_MAX, W), t0)
    del x
    exp = None
    for r in range(p):
        blk = gen_f64(0xC4 + r, n)[rank * per:(rank + 1) * per].clone()
        exp = blk if exp is None else torch.maximum(exp, blk)
    torch.cuda.synchronize()
    if not torch.equal(y.view(torch.int64), exp.view(torch.int64)):
        fails.append(f"c4: {(y != exp).sum().item()} elements differ")
else:
    n = 1 << 26                                   # 512 MiB of uint64 per rank
    x = gen_u64(0xC5 + rank, n)
    y = torch.empty_like(x)
    torch.cuda.synchronize()
    req = ctypes.c_int()
    t0 = time.perf_counter()
    rc = L.MPI_Iallreduce(x.data_ptr(), y.data_ptr(), n, C.MPI_UINT64_T, C.MPI_BAND, W, ctypes.byref(req))
    a = np.random.default_rng(rank).standard_normal(1 << 22)
    for _ in range(20):                           # host work while the reduction runs
        a = 1.0001 * a + 0.5
    t_host = time.perf_counter() - t0
    rc = rc or L.MPI_Wait(ctypes.byref(req), ctypes.c_void_p(1))
    done(f"c5 iallreduce (host work {t_host:.3f}s)", rc, t0)
    exp = gen_u64(0xC5, n)
    for r in range(1, p):
        exp &= gen_u64(0xC5 + r, n)
    torch.cuda.synchronize()
    if not torch.equal(y, exp):
        fails.append(f"c5: {(y != exp).sum().item()} elements differ")
    if torch.equal(exp, torch.zeros_like(exp)) or torch.equal(exp, torch.full_like(exp, -1)):
        fails.append("c5: trivial data")
L.msx_engine_transport.restype = ctypes.c_char_p
print("TRANSPORT", L.msx_engine_transport().decode(), flush=True)
print("RESULT", rank, p, len(fails), fails[:5], flush=True)
L.MPI_Finalize()
'''


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _run(cfg, p, one_per_gpu=False, transport=None, extra=None):
    port = _free_port()
    procs = []
    for r in range(p):
        env = dict(os.environ)
        env.update({"MSX_SIZE": str(p), "MSX_RANK": str(r), "MSX_DEVICE": str(r) if one_per_gpu else "0",
                    "FULL_CFG": cfg, "MSX_BOOTSTRAP_PORT": str(port), "MSX_BOOTSTRAP_ADDR": "127.0.0.1",
                    "MSX_BOOTSTRAP_TIMEOUT": "120"})
        if transport:
            env["MSX_TRANSPORT"] = transport
            env["MSX_FLAG_TIMEOUT_MS"] = "60000"
        env.update(extra or {})
        procs.append(subprocess.Popen([sys.executable, "-c", f"REPO={REPO!r}\n" + textwrap.dedent(WORKER)],
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env))
    results = []
    deadline = time.monotonic() + (150 if p <= 3 else 220)
    for pr in procs:
        try:
            o, e = pr.communicate(timeout=max(1.0, deadline - time.monotonic()))
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            o, e = pr.communicate()
        results.append((pr.returncode, o, e))
    lines, ok = [], True
    for r, (rc, o, e) in enumerate(results):
        res = [l for l in o.splitlines() if l.startswith("RESULT")]
        if rc != 0 or not res:
            ok = False
            lines.append(f"rank {r}: rc={rc} {(o + e)[-1500:]}")
        else:
            ok = ok and res[0].split()[3] == "0"
            lines.append(res[0])
    assert ok, "\n".join(lines)        # every rank's line, not just the first failing one
    return [[l.split()[1] for l in o.splitlines() if l.startswith("TRANSPORT")] for _, o, _ in results]


# Ranks sharing the one GPU take the host-barrier schedules by default since
# round 4; `flags` forces the GPU-flag ones (the pipelined
# two-step allreduce, pipelined reduce_scatter rounds) that one rank per GPU
# runs by default.
@pytest.mark.parametrize("cfg,p,sched", [("c3", 2, "default"), ("c3", 3, "default"), ("c4", 2, "default"),
                                         ("c5", 2, "default"), ("c3", 8, "default"), ("c4", 8, "default"),
                                         ("c5", 8, "default"), ("c3", 2, "flags"), ("c3", 3, "flags"),
                                         ("c4", 2, "flags"), ("c5", 2, "flags"), ("c3", 8, "flags"),
                                         ("c4", 8, "flags")])
def test_baseline_config_full_size(cfg, p, sched):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _run(cfg, p, extra={"MSX_TWO_STEP_MAX": str(1 << 62)} if sched == "flags" else None)


# The configs at their own layout: 8 ranks, ONE PER GPU (MSX_DEVICE = rank),
# on both data planes -- IPC windows written over xGMI (the exchange sites of
# reduce.cpp:3973,4047 for c3, :1126 for c4, :4421-4472,4549-4577 for c5) and
# RCCL send/recv -- checked against the same 8-leaf reference trees.  Skipped
# below 8 GPUs (the one-GPU box); the driver's 8-GPU node runs them.
# `sched`: the default for distinct GPUs (GPU-flag two-step up to 256 MiB,
# host barriers above), the host-barrier schedules only (MSX_TWO_STEP_MAX=0)
# and the opt-in GPU-flag pipeline at every size, so a failure tells the
# schedule from the data plane.
SCHED_ENV = {"default": None, "host_barrier": {"MSX_TWO_STEP_MAX": "0"},
             "pipeline": {"MSX_TWO_STEP_MAX": str(1 << 62)}}


@pytest.mark.parametrize("sched", ["default", "host_barrier", "pipeline"])
@pytest.mark.parametrize("transport", ["ipc", "rccl"])
@pytest.mark.parametrize("cfg", ["c3", "c4", "c5"])
def test_baseline_config_one_rank_per_gpu(cfg, transport, sched):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    if torch.cuda.device_count() < 8:
        pytest.skip("needs 8 GPUs (one rank per GPU, the configs' layout)")
    used = _run(cfg, 8, one_per_gpu=True, transport=transport,
                extra=SCHED_ENV[sched])
    assert all(u == [transport] for u in used), used
