"""Probe: latency of small MPI_Allreduce / MPI_Reduce (fp32 SUM, device
buffers) with P ranks on this box, OSU style (back-to-back calls after one
barrier, averaged).  Prints one JSON line on rank 0.  A measurement, not a test.
usage: MSX_SIZE=P MSX_RANK=r MSX_DEVICE=0 ... python scripts/small_coll_probe.py"""
import ctypes
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "microsoft-mpi_amd"))
import msx  # noqa: E402

L = msx.init(errors_return=True)
C = msx.C
r_, s_ = ctypes.c_int(), ctypes.c_int()
L.MPI_Comm_rank(C.MPI_COMM_WORLD, ctypes.byref(r_))
L.MPI_Comm_size(C.MPI_COMM_WORLD, ctypes.byref(s_))
rank, p = r_.value, s_.value
out = {"ranks": p, "spin_us": os.environ.get("MSX_SYNC_SPIN_US")}
for nbytes in (8, 4096, 65536):
    m = max(1, nbytes // 4)
    a = torch.ones(m, device="cuda")
    b = torch.zeros(m, device="cuda")
    torch.cuda.synchronize()
    for _ in range(20):
        L.MPI_Allreduce(a.data_ptr(), b.data_ptr(), m, C.MPI_FLOAT, C.MPI_SUM, C.MPI_COMM_WORLD)
    ts = []
    for _ in range(5):
        L.MPI_Barrier(C.MPI_COMM_WORLD)
        t0 = time.perf_counter()
        for _ in range(200):
            L.MPI_Allreduce(a.data_ptr(), b.data_ptr(), m, C.MPI_FLOAT, C.MPI_SUM, C.MPI_COMM_WORLD)
        ts.append((time.perf_counter() - t0) / 200)
    ok = bool(torch.all(b == p).item())
    out[f"allreduce_{nbytes}B_us"] = [round(sorted(ts)[2] * 1e6, 2), ok]
    ts = []
    for _ in range(5):
        L.MPI_Barrier(C.MPI_COMM_WORLD)
        t0 = time.perf_counter()
        for _ in range(200):
            L.MPI_Reduce(a.data_ptr(), b.data_ptr(), m, C.MPI_FLOAT, C.MPI_SUM, 0, C.MPI_COMM_WORLD)
        ts.append((time.perf_counter() - t0) / 200)
    out[f"reduce_{nbytes}B_us"] = round(sorted(ts)[2] * 1e6, 2)
# host (pageable) buffers: the common case of a CPU application
import numpy as np  # noqa: E402
for nbytes in (8, 4096, 65536):
    m = max(1, nbytes // 4)
    ha = np.ones(m, np.float32)
    hb = np.zeros(m, np.float32)
    for _ in range(20):
        L.MPI_Allreduce(ha.ctypes.data, hb.ctypes.data, m, C.MPI_FLOAT, C.MPI_SUM, C.MPI_COMM_WORLD)
    ts = []
    for _ in range(5):
        L.MPI_Barrier(C.MPI_COMM_WORLD)
        t0 = time.perf_counter()
        for _ in range(200):
            L.MPI_Allreduce(ha.ctypes.data, hb.ctypes.data, m, C.MPI_FLOAT, C.MPI_SUM, C.MPI_COMM_WORLD)
        ts.append((time.perf_counter() - t0) / 200)
    out[f"host_allreduce_{nbytes}B_us"] = [round(sorted(ts)[2] * 1e6, 2), bool((hb == p).all())]
    hc = np.ones(m, np.float32)
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        for _ in range(200):
            L.MPI_Reduce_local(ha.ctypes.data, hc.ctypes.data, m, C.MPI_FLOAT, C.MPI_SUM)
        ts.append((time.perf_counter() - t0) / 200)
    out[f"host_reduce_local_{nbytes}B_us"] = round(sorted(ts)[2] * 1e6, 2)
    da = torch.ones(m, device="cuda")
    db = torch.ones(m, device="cuda")
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        for _ in range(200):
            L.MPI_Reduce_local(da.data_ptr(), db.data_ptr(), m, C.MPI_FLOAT, C.MPI_SUM)
        ts.append((time.perf_counter() - t0) / 200)
    out[f"device_reduce_local_{nbytes}B_us"] = round(sorted(ts)[2] * 1e6, 2)
if rank == 0:
    print(json.dumps(out), flush=True)
L.MPI_Finalize()
