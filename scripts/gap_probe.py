"""Gapped-access probe (measurement only): is the 2x HBM write traffic of the
16-B-block vector's unpack (k_dt_pack<16,true,true,true>: 16 B written of
every 32 B) the kernel's, or the access pattern's?  Times, over the same
256 MiB span: a contiguous store and load (HBM probe modes 1 / 3), the gapped
store / load of 16 B of every 32 B (modes 6 / 7), and MPI_Unpack / MPI_Pack of
that vector type through msx_unpack_dev / msx_pack_dev.  Run under
`rocprofv3 --pmc FETCH_SIZE` and `--pmc WRITE_SIZE` (separate passes) to read
each kernel's HBM bytes per launch."""
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "microsoft-mpi_amd"))
import torch  # noqa: E402

import msx  # noqa: E402

L = msx.init(errors_return=True)
C = msx.C
stream = torch.cuda.Stream()
torch.cuda.set_stream(stream)
sp = ctypes.c_void_p(stream.cuda_stream)
NB = 256 << 20
a = torch.randn(NB // 4, device="cuda")
b = torch.randn(NB // 4, device="cuda")
packed = torch.empty(NB // 2, dtype=torch.uint8, device="cuda")
t = ctypes.c_int()
assert L.MPI_Type_vector(NB // 32, 4, 8, C.MPI_FLOAT, ctypes.byref(t)) == 0
assert L.MPI_Type_commit(ctypes.byref(t)) == 0
torch.cuda.synchronize()


def timed(fn, reps=10):
    ts = []
    for _ in range(3):
        fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            assert fn() == 0, msx.last_error()
        e1.record(stream)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / reps)
    return sorted(ts)[1] * 1e3


out = {}
for label, mode, touched in (("store_contiguous_256MiB", 1, NB), ("load_contiguous_256MiB", 3, NB),
                             ("store_16of32B_span256MiB", 6, NB // 2), ("load_16of32B_span256MiB", 7, NB // 2)):
    us = timed(lambda: L.msx_probe_hbm(mode, a.data_ptr(), b.data_ptr(), NB, sp))
    out[label] = {"us": round(us, 1), "algorithmic_bytes": touched, "GB_s": round(touched / us / 1e3, 1)}
for label, fn, x, y in (("unpack_vector16of32", L.msx_unpack_dev, packed, b), ("pack_vector16of32", L.msx_pack_dev, b, packed)):
    us = timed(lambda: fn(x.data_ptr(), 1, t.value, y.data_ptr(), sp))
    out[label] = {"us": round(us, 1), "algorithmic_bytes": NB, "GB_s": round(NB / us / 1e3, 1)}
print(json.dumps(out), flush=True)
