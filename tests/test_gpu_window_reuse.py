"""GPU: a freed communicator's uncached window is kept and reused, never freed.

Each communicator's engine window is uncached device memory
(hipDeviceMallocUncached) that the peers map over IPC.  On this ROCm stack,
once such memory has been used and freed, later allocations in the same process
can read back wrong data (scripts/va_reuse_probe.py: torch.equal(a, a.clone())
on fresh tensors false in 4-30 of 96 cases per variant after uncached buffers
were used and freed; 0 with the buffers kept, 0 with plain buffers freed;
profiles/r06/va_reuse/).  The library keeps every uncached block for the life of
the process (msx_transport.cpp uc_pool) and keeps imported peer windows mapped.
Two ranks on one GPU create, use and free communicators: the device memory of a
freed communicator's window stays allocated, the next communicator's window
takes it (no further allocation), and every allreduce is exact.
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
CHUNK = 64 << 20          # window = 2 x CHUNK + flags per rank

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
n = 3 << 20
x = lambda r, it: ((np.arange(n, dtype=np.int64) * 7 + r * 131 + it) % 65521).astype(np.int32)
send = torch.zeros(n, dtype=torch.int32, device="cuda"); recv = torch.zeros_like(send)
def free_mem():
    L.MPI_Barrier(C.MPI_COMM_WORLD)       # both ranks' allocations done
    torch.cuda.synchronize()
    f = torch.cuda.mem_get_info()[0]
    L.MPI_Barrier(C.MPI_COMM_WORLD)
    return f
mem = []
for it in range(4):
    dup = ctypes.c_int()
    if L.MPI_Comm_dup(C.MPI_COMM_WORLD, ctypes.byref(dup)):
        fails.append(f"dup {it}: {msx.last_error()}"); break
    send.copy_(torch.from_numpy(x(rank, it))); recv.zero_(); torch.cuda.synchronize()
    if L.MPI_Allreduce(send.data_ptr(), recv.data_ptr(), n, C.MPI_INT, C.MPI_SUM, dup.value):
        fails.append(f"allreduce {it}: {msx.last_error()}")
    exp = sum(x(r, it).astype(np.int64) for r in range(p)).astype(np.int32)
    if not np.array_equal(recv.cpu().numpy(), exp):
        fails.append(f"allreduce {it} result")
    in_use = free_mem()
    if L.MPI_Comm_free(ctypes.byref(dup)):
        fails.append(f"free {it}: {msx.last_error()}")
    mem.append((in_use, free_mem()))
print("RESULT", rank, p, len(fails), fails[:4], flush=True)
print("MEM", " ".join(f"{a}:{b}" for a, b in mem), flush=True)
L.MPI_Finalize()
'''


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_freed_communicator_windows_are_kept_and_reused():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    p = 2
    port = _free_port()
    procs = []
    for r in range(p):
        env = dict(os.environ)
        env.update({"MSX_SIZE": str(p), "MSX_RANK": str(r), "MSX_DEVICE": "0",
                    "MSX_BOOTSTRAP_PORT": str(port), "MSX_BOOTSTRAP_ADDR": "127.0.0.1",
                    "MSX_BOOTSTRAP_TIMEOUT": "180", "MSX_CHUNK_BYTES": str(CHUNK)})
        procs.append(subprocess.Popen([sys.executable, "-c", f"REPO={REPO!r}\n" + textwrap.dedent(WORKER)],
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env))
    outs = []
    for pr in procs:
        try:
            o, e = pr.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            pr.kill()
            o, e = pr.communicate()
        assert pr.returncode == 0, (o + e)[-3000:]
        line = [l for l in o.splitlines() if l.startswith("RESULT")]
        assert line, (o + e)[-3000:]
        assert line[0].split()[3] == "0", line[0]
        outs.append(o)
    mem = [tuple(int(v) for v in pair.split(":"))
           for pair in [l for l in outs[0].splitlines() if l.startswith("MEM")][0].split()[1:]]
    window = 2 * CHUNK
    for k, (in_use, after_free) in enumerate(mem):
        # freeing the communicator gives no window memory back (both ranks' windows kept)
        assert after_free - in_use < window // 2, (k, mem)
        if k:
            # the next communicator's windows are the kept ones: no new window allocation
            assert mem[k - 1][1] - in_use < window // 2, (k, mem)
