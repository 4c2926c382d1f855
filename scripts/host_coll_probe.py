"""Probe: MPI_Allreduce (fp32 SUM) on host buffers -- pageable, pinned by the
user, and device-resident for reference -- with P ranks of this box.  Prints
one JSON line per rank 0.  A measurement, not a test.
usage: MSX_SIZE=P MSX_RANK=r MSX_DEVICE=0 ... python scripts/host_coll_probe.py MiB"""
import ctypes
import json
import os
import sys
import time

import numpy as np
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
n = int(float(sys.argv[1]) * (1 << 20)) // 4
x = (np.arange(n, dtype=np.int64) % 17 - 8 + rank).astype(np.float32)
exp = sum((np.arange(n, dtype=np.int64) % 17 - 8 + r).astype(np.float32) for r in range(p))
out = {}


def run(label, sp, rp, check):
    ts = []
    for _ in range(4):
        L.MPI_Barrier(C.MPI_COMM_WORLD)
        t0 = time.perf_counter()
        rc = L.MPI_Allreduce(sp, rp, n, C.MPI_FLOAT, C.MPI_SUM, C.MPI_COMM_WORLD)
        ts.append(time.perf_counter() - t0)
        assert rc == 0, msx.last_error()
    t = sorted(ts[1:])[1]
    out[label] = {"ms": round(t * 1e3, 2), "algbw_GB_s": round(n * 4 / t / 1e9, 2), "correct": check()}


hr = np.empty_like(x)
run("pageable", x.ctypes.data, hr.ctypes.data, lambda: bool(np.array_equal(hr, exp)))
ps = torch.from_numpy(x.copy()).pin_memory()
pr = torch.empty_like(ps).pin_memory()
run("pinned", ps.data_ptr(), pr.data_ptr(), lambda: bool(np.array_equal(pr.numpy(), exp)))
ds = torch.from_numpy(x).cuda()
dr = torch.empty_like(ds)
torch.cuda.synchronize()
run("device", ds.data_ptr(), dr.data_ptr(), lambda: bool(np.array_equal(dr.cpu().numpy(), exp)))
st = (ctypes.c_double * 7)()
L.msx_engine_stats(st, 7, 0)
out["phase_s_total"] = [round(v, 4) for v in st]
if rank == 0:
    print(json.dumps({"ranks": p, "MiB": float(sys.argv[1]), "pin_min": os.environ.get("MSX_HOST_PIN_MIN"), **out}),
          flush=True)
L.MPI_Finalize()
