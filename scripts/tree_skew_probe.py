"""Probe: does the p-source combine (k_tree) lose HBM bandwidth when its
sources sit a power of two apart (the IN sub-slots of a window are Q = C/p
bytes apart)?  Times msx_reduce_tree_dev over p = 8 sources of 32 MiB each,
placed at stride 32 MiB (the bench's layout) and at strides skewed by a few
KiB, and prints one JSON line.  GPU only; a measurement, not a test."""
import ctypes
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "microsoft-mpi_amd"))
import msx  # noqa: E402

L = msx.init(errors_return=True)
C = msx.C
dev = torch.device("cuda:0")
stream = torch.cuda.Stream(dev)
sp = ctypes.c_void_p(stream.cuda_stream)
p, m = 8, (32 << 20) // 4
res = {}
a = torch.empty(p * (m * 4 + (1 << 20)), dtype=torch.uint8, device=dev)
a.view(torch.float32).uniform_(-1, 1)
b = torch.empty(m * 4, dtype=torch.uint8, device=dev)
torch.cuda.synchronize()
for skew in (0, 256, 4096, 4096 + 256, 65536 + 4096, 1 << 20):
    stride = m * 4 + skew
    srcs = (ctypes.c_void_p * p)(*[a.data_ptr() + r * stride for r in range(p)])
    ts = []
    for _ in range(5):
        for _ in range(2):
            L.msx_reduce_tree_dev(srcs, p, b.data_ptr(), m, C.MPI_FLOAT, C.MPI_SUM, sp)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(20):
            rc = L.msx_reduce_tree_dev(srcs, p, b.data_ptr(), m, C.MPI_FLOAT, C.MPI_SUM, sp)
            assert rc == 0, rc
        e1.record(stream)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / 20)
    ms = sorted(ts)[2]
    res[f"skew{skew}"] = {"us": round(ms * 1e3, 1), "GB_s": round((p + 1) * m * 4 / ms / 1e6, 1)}
    print(f"skew {skew}: {res[f'skew{skew}']}", flush=True)
print(json.dumps(res))
