#!/usr/bin/env python3
"""One rank of a collective timing probe (fp32 SUM, device buffers).
Usage: MSX_SIZE/MSX_RANK/... python3 scripts/allreduce_probe.py NBYTES ITERS [allreduce|rsb|reduce|scan]
NBYTES is the per-rank message (allreduce, reduce) or the whole input
(reduce_scatter_block: NBYTES / p per block)."""
import ctypes, os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "microsoft-mpi_amd"))
import torch
import msx
L = msx.init(errors_return=True)
C = msx.C
r_ = ctypes.c_int(); L.MPI_Comm_rank(C.MPI_COMM_WORLD, ctypes.byref(r_))
nbytes, iters = int(sys.argv[1]), int(sys.argv[2])
kind = sys.argv[3] if len(sys.argv) > 3 else "allreduce"
p = int(os.environ["MSX_SIZE"])
n = nbytes // 4
a = torch.ones(n, device="cuda"); b = torch.zeros(n, device="cuda"); torch.cuda.synchronize()
W = C.MPI_COMM_WORLD
if kind == "allreduce":
    call = lambda: L.MPI_Allreduce(a.data_ptr(), b.data_ptr(), n, C.MPI_FLOAT, C.MPI_SUM, W)
    check = lambda: bool(torch.all(b == float(p)).item())
elif kind == "rsb":
    call = lambda: L.MPI_Reduce_scatter_block(a.data_ptr(), b.data_ptr(), n // p, C.MPI_FLOAT, C.MPI_SUM, W)
    check = lambda: bool(torch.all(b[: n // p] == float(p)).item())
elif kind == "scan":
    L.MPI_Scan.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]
    call = lambda: L.MPI_Scan(a.data_ptr(), b.data_ptr(), n, C.MPI_FLOAT, C.MPI_SUM, W)
    check = lambda: bool(torch.all(b == float(r_.value + 1)).item())
else:
    call = lambda: L.MPI_Reduce(a.data_ptr(), b.data_ptr(), n, C.MPI_FLOAT, C.MPI_SUM, 0, W)
    check = lambda: r_.value != 0 or bool(torch.all(b == float(p)).item())
for _ in range(3):
    call()
L.MPI_Barrier(W)
t0 = time.perf_counter()
for _ in range(iters):
    call()
t = (time.perf_counter() - t0) / iters
print(f"rank {r_.value} {kind} bytes {nbytes} us {t * 1e6:.1f} ok {check()}", flush=True)
L.MPI_Finalize()
