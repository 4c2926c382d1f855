"""GPU: a rank that never arrives ends the job with a diagnosis, not a hang.

Every cross-rank wait in the engine is bounded (GPU flag waits by
MSX_FLAG_TIMEOUT_MS, measured on the 100 MHz s_memrealtime clock inside the
kernel; host barriers by MSX_BOOTSTRAP_TIMEOUT) and names what it waited for.
MSX_TEST_DROP_FLAGS=<rank>:<seq> (test-only fault injection,
msx_transport.cpp fault_drop_flags) makes <rank> skip its arrival-flag posts
of flag-synchronised call <seq>, so its peer's wait must run out.

Two ranks share the box's GPU; the dropped call is a 4 KiB device allreduce
(the single-kernel flag path).
* MPI_ERRORS_RETURN: rank 0's MPI_Allreduce returns an error and
  msx_last_error() carries `flag timeout: op=allreduce rank=0 phase=arrival
  peer=1 ...`; both ranks then meet in MPI_Barrier and exit cleanly.
* MPI_ERRORS_ARE_FATAL (the default handler): rank 0 exits non-zero with that
  line on stderr; rank 1, left waiting at the next barrier, exits non-zero
  with `wait timeout: op=barrier rank=1 phase=host_barrier peer=0 ...`."""
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
import ctypes, os, sys
sys.path.insert(0, os.path.join(REPO, "microsoft-mpi_amd")); sys.path.insert(0, REPO)
import torch
import msx
C = msx.C
RET = os.environ["FAULT_MODE"] == "return"
L = msx.init(errors_return=RET)
r_ = ctypes.c_int()
L.MPI_Comm_rank(C.MPI_COMM_WORLD, ctypes.byref(r_))
rank = r_.value
sb = torch.full((1024,), float(rank + 1), dtype=torch.float32, device="cuda")
rb = torch.zeros(1024, dtype=torch.float32, device="cuda")
torch.cuda.synchronize()
rc = L.MPI_Allreduce(sb.data_ptr(), rb.data_ptr(), 1024, C.MPI_FLOAT, C.MPI_SUM, C.MPI_COMM_WORLD)
print("ALLREDUCE", rank, rc, msx.last_error() if rc else "", flush=True)
rc2 = L.MPI_Barrier(C.MPI_COMM_WORLD)
print("BARRIER", rank, rc2, msx.last_error() if rc2 else "", flush=True)
sys.stdout.flush()
os._exit(0)
'''


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _run(mode, bar_timeout):
    port = _free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ)
        env.update({"MSX_SIZE": "2", "MSX_RANK": str(r), "MSX_DEVICE": "0",
                    "MSX_BOOTSTRAP_PORT": str(port), "MSX_BOOTSTRAP_ADDR": "127.0.0.1",
                    "MSX_BOOTSTRAP_TIMEOUT": str(bar_timeout), "MSX_FLAG_TIMEOUT_MS": "3000",
                    "MSX_TEST_DROP_FLAGS": "1:1", "FAULT_MODE": mode})
        env.pop("MSMPI_FORCE_ASYNC_WORKFLOW", None)
        procs.append(subprocess.Popen([sys.executable, "-c",
                                       f"REPO={REPO!r}\n" + textwrap.dedent(WORKER)],
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env))
    out = []
    for pr in procs:
        try:
            o, e = pr.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            pr.kill()
            o, e = pr.communicate()
            o += "\n[killed by the test: no diagnosis within 240 s]"
        out.append((pr.returncode, o, e))
    return out


def test_dropped_arrival_returns_structured_error():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    (rc0, o0, e0), (rc1, o1, e1) = _run("return", 120)
    assert rc0 == 0 and rc1 == 0, (o0 + e0 + o1 + e1)[-3000:]
    a0 = [l for l in o0.splitlines() if l.startswith("ALLREDUCE")]
    assert a0 and a0[0].split()[2] != "0", (o0 + e0)[-2000:]
    assert "flag timeout: op=allreduce rank=0 phase=arrival peer=1 seq=1 limit_s=3.0" in a0[0], a0[0]
    # rank 1's own flag wait was satisfied (rank 0 posted): its call succeeds
    a1 = [l for l in o1.splitlines() if l.startswith("ALLREDUCE")]
    assert a1 and a1[0].split()[2] == "0", (o1 + e1)[-2000:]
    for o in (o0, o1):
        b = [l for l in o.splitlines() if l.startswith("BARRIER")]
        assert b and b[0].split()[2] == "0", o[-2000:]


def test_dropped_arrival_is_fatal_with_diagnosis():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    t0 = time.monotonic()
    (rc0, o0, e0), (rc1, o1, e1) = _run("fatal", 30)
    elapsed = time.monotonic() - t0
    assert rc0 != 0, (o0 + e0)[-2000:]
    assert "flag timeout: op=allreduce rank=0 phase=arrival peer=1" in o0 + e0, (o0 + e0)[-2000:]
    assert not [l for l in o0.splitlines() if l.startswith("BARRIER")], o0[-2000:]
    assert rc1 != 0, (o1 + e1)[-2000:]
    assert "wait timeout: op=barrier rank=1 phase=host_barrier peer=0" in o1 + e1, (o1 + e1)[-2000:]
    assert elapsed < 200, elapsed
