"""Probe: IPC-map torch and hipMalloc buffers of growing size between 2 ranks on one GPU."""
import ctypes, os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "microsoft-mpi_amd"))
import torch, msx
C = msx.C
L = msx.init()
r = ctypes.c_int(); L.MPI_Comm_rank(C.MPI_COMM_WORLD, ctypes.byref(r))
for mb in [int(x) for x in sys.argv[1:]]:
    n = mb * (1 << 20) // 4
    a = torch.ones(n, device="cuda") * (r.value + 1)
    b = torch.empty_like(a)
    torch.cuda.synchronize()
    t0 = time.time()
    rc = L.MPI_Allreduce(a.data_ptr(), b.data_ptr(), n, C.MPI_FLOAT, C.MPI_SUM, C.MPI_COMM_WORLD)
    print(f"rank {r.value} {mb} MiB rc={rc} {time.time()-t0:.3f}s ok={bool((b == 3).all())}", flush=True)
L.MPI_Finalize()
