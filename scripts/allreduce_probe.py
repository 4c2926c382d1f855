#!/usr/bin/env python3
"""One rank of an allreduce timing probe (fp32 SUM, device buffers).
Usage: MSX_SIZE/MSX_RANK/... python3 scripts/allreduce_probe.py NBYTES ITERS"""
import ctypes, os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "microsoft-mpi_amd"))
import torch
import msx
L = msx.init(errors_return=True)
C = msx.C
r_ = ctypes.c_int(); L.MPI_Comm_rank(C.MPI_COMM_WORLD, ctypes.byref(r_))
nbytes, iters = int(sys.argv[1]), int(sys.argv[2])
n = nbytes // 4
a = torch.ones(n, device="cuda"); b = torch.zeros(n, device="cuda"); torch.cuda.synchronize()
for _ in range(3):
    L.MPI_Allreduce(a.data_ptr(), b.data_ptr(), n, C.MPI_FLOAT, C.MPI_SUM, C.MPI_COMM_WORLD)
L.MPI_Barrier(C.MPI_COMM_WORLD)
t0 = time.perf_counter()
for _ in range(iters):
    L.MPI_Allreduce(a.data_ptr(), b.data_ptr(), n, C.MPI_FLOAT, C.MPI_SUM, C.MPI_COMM_WORLD)
t = (time.perf_counter() - t0) / iters
print(f"rank {r_.value} bytes {nbytes} us {t * 1e6:.1f} ok {bool(torch.all(b == float(int(os.environ['MSX_SIZE']))).item())}",
      flush=True)
L.MPI_Finalize()
