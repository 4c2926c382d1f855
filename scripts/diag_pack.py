import ctypes, sys
sys.path.insert(0, "microsoft-mpi_amd")
import torch, msx
L = msx.init(errors_return=True); C = msx.C
for n in (1 << 20, 1 << 24, 1 << 26, 1 << 28):
    x = torch.randn(n, device="cuda")
    t = ctypes.c_int()
    assert L.MPI_Type_vector(n // 2, 1, 2, C.MPI_FLOAT, ctypes.byref(t)) == 0
    assert L.MPI_Type_commit(ctypes.byref(t)) == 0
    out = torch.full((n // 2,), 7.0, device="cuda")
    torch.cuda.synchronize()
    pos = ctypes.c_int(0)
    rc = L.MPI_Pack(x.data_ptr(), 1, t.value, out.data_ptr(), 2 * n, ctypes.byref(pos), C.MPI_COMM_WORLD)
    torch.cuda.synchronize()
    bad = (out != x[::2]).nonzero().flatten()
    print(n, rc, pos.value, bad.numel(), bad[:5].tolist(), bad[-5:].tolist() if bad.numel() else [], flush=True)
    if bad.numel():
        i = bad[0].item()
        print("  got", out[i:i+4].tolist(), "want", x[::2][i:i+4].tolist(), "x", x[2*i-2:2*i+6].tolist())
    L.MPI_Type_free(ctypes.byref(t))
