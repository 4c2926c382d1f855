"""Derived-target accumulate (measurement only): MPI_Accumulate fp32 SUM of a
contiguous origin into a self-targeted device window through a vector target
type (16-B blocks at a 32-B stride), i.e. k_dt_acc, in its grid-stride form
(msx_tune_pack 1) and its one-wave tile form (2), window sizes ACC_MIB
(default 256, 1024) MiB, interleaved rounds, host clock around K calls inside
one fence epoch.  Checked against torch.  Prints one JSON line."""
import ctypes
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "microsoft-mpi_amd"))
import torch  # noqa: E402

import msx  # noqa: E402

L = msx.init(errors_return=True)
C = msx.C
out = {}
for mib in [int(x) for x in os.environ.get("ACC_MIB", "256,1024").split(",")]:
    nf = mib << 18
    win = torch.randn(nf, device="cuda")
    src = torch.randn(nf // 2, device="cuda")
    vt = ctypes.c_int()
    assert L.MPI_Type_vector(nf // 8, 4, 8, C.MPI_FLOAT, ctypes.byref(vt)) == 0
    assert L.MPI_Type_commit(ctypes.byref(vt)) == 0
    w = ctypes.c_int()
    torch.cuda.synchronize()
    assert L.MPI_Win_create(win.data_ptr(), nf * 4, 4, C.MPI_INFO_NULL, C.MPI_COMM_WORLD, ctypes.byref(w)) == 0
    for mode in (1, 2):                                   # parity of both forms
        assert L.msx_tune_pack(mode) == 0
        want = win.view(-1, 8).clone()
        want[:, :4] += src.view(-1, 4)
        torch.cuda.synchronize()
        assert L.MPI_Win_fence(0, w) == 0
        assert L.MPI_Accumulate(src.data_ptr(), nf // 2, C.MPI_FLOAT, 0, 0, 1, vt.value, C.MPI_SUM, w) == 0, \
            msx.last_error()
        assert L.MPI_Win_fence(0, w) == 0
        torch.cuda.synchronize()
        out[f"{mib}/mode{mode}/correct"] = bool(torch.equal(win.view(-1, 8), want))
        del want
    K = 10
    for rnd in range(3):
        for mode, name in ((1, "grid_stride"), (2, "tile")):
            assert L.msx_tune_pack(mode) == 0
            assert L.MPI_Win_fence(0, w) == 0
            t0 = time.perf_counter()
            for _ in range(K):
                L.MPI_Accumulate(src.data_ptr(), nf // 2, C.MPI_FLOAT, 0, 0, 1, vt.value, C.MPI_SUM, w)
            assert L.MPI_Win_fence(0, w) == 0
            torch.cuda.synchronize()
            us = (time.perf_counter() - t0) / K * 1e6
            out.setdefault(f"{mib}/{name}_us_per_call", []).append(round(us, 1))
    assert L.msx_tune_pack(0) == 0
    assert L.MPI_Win_free(ctypes.byref(w)) == 0
    L.MPI_Type_free(ctypes.byref(vt))
    del win, src
    torch.cuda.empty_cache()
print(json.dumps(out), flush=True)
