"""Combine rate for mutually misaligned operands (measurement only): 256 MiB
fp32 / fp64 / int8 MPI_SUM with `in` offset from 16-byte alignment by 0..12
bytes (element-aligned) while `inout` stays aligned, and both offset alike."""
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
sp = ctypes.c_void_p(stream.cuda_stream)
NB = 256 << 20
a = torch.empty(NB + 64, dtype=torch.uint8, device="cuda")
b = torch.empty(NB + 64, dtype=torch.uint8, device="cuda")
a.view(torch.float32)[:].uniform_(-1, 1)
b.view(torch.float32)[:].uniform_(-1, 1)
torch.cuda.synchronize()
out = {}
MODES = {"dpp": 0, "bpermute": 1, "dpp_skewed_grid": 2}


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
    return sorted(ts)[1]


for dtn, esz in (("MPI_FLOAT", 4), ("MPI_DOUBLE", 8), ("MPI_INT8_T", 1), ("MPI_INT", 4)):
    dt = getattr(C, dtn)
    for oa, ob in ((0, 0), (esz, 0), (2 * esz, 0), (4 if esz < 8 else 8, 4 if esz < 8 else 8), (12 if esz == 4 else esz, 0)):
        if oa % esz or ob % esz:
            continue
        n = (NB - 16) // esz
        for mname, mode in MODES.items():     # the realigning kernel's cross-lane move, A/B in one process
            if (oa - ob) % 16 == 0 and mode:
                continue                       # aligned pairs do not use it
            L.msx_tune_shift(mode)
            ms = timed(lambda: L.msx_reduce_local_dev(a.data_ptr() + oa, b.data_ptr() + ob, n, dt, C.MPI_SUM, sp))
            key = f"{dtn}/in+{oa}/io+{ob}" + ("" if (oa - ob) % 16 == 0 else f"/{mname}")
            out[key] = {"us": round(ms * 1e3, 1), "GB_s": round(3 * n * esz / ms / 1e6, 1)}
L.msx_tune_shift(0)
print(json.dumps(out), flush=True)
