"""p = 8 fp32 SUM collective tree below the Infinity Cache bound (measurement
only): the default there (tuning mode 4: plain loads, 256-lane XCD-contiguous
tiles) against the DRAM-regime form (mode 15: non-temporal loads, 64-lane
workgroups in dispatch order), per source size, in two conditions:
  fresh -- every launch follows a rewrite of all 8 sources by the engine's
           copy kernel (what the scatter pushes leave behind), timed alone;
  reread -- back-to-back launches over the same sources.
Sources in uncached device memory (the windows' type), HIP events, median.
Usage: python scripts/tree_fresh_probe.py [MiB per source,...] -> one JSON line."""
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
sizes = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "4,8,16,24,32").split(",")]
skew = 68 << 10


def alloc(nbytes):
    q = ctypes.c_void_p()
    assert L.msx_probe_alloc(nbytes, 1, ctypes.byref(q)) == 0, msx.last_error()
    return q.value


def ev(fn, k=1):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(k):
        fn()
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / k


res = {"p": 8, "memory": "uncached (the windows' type)", "modes": {"4": "default below tree_nt_min",
                                                                       "15": "DRAM-regime form"}}
maxn = max(sizes) << 18
slot = maxn * 4 + skew
base = alloc(8 * slot)
srcs = [base + k * slot for k in range(8)]
fill = torch.rand(maxn, device="cuda")
out_t = torch.empty(maxn, device="cuda")
torch.cuda.synchronize()
for mib in sizes:
    n = mib << 18
    arr = (ctypes.c_void_p * 16)(*[srcs[k // 2] if k % 2 == 0 else srcs[k // 2] for k in range(16)])
    refill = lambda: [L.msx_probe_hbm(4, fill.data_ptr(), ctypes.c_void_p(s), n * 4, sp) for s in srcs]
    row, outs = {}, {}
    for rnd in range(3):
        for mode in (4, 15):
            assert L.msx_tune_tree(mode, 0) == 0
            call = lambda: L.msx_reduce_tree_spec_dev(arr, 8, 0, 8, 0, out_t.data_ptr(), n, C.MPI_FLOAT, C.MPI_SUM, sp)
            refill()
            assert call() == 0, msx.last_error()
            torch.cuda.synchronize()
            outs[mode] = out_t[:n].clone()
            fresh = []
            for _ in range(9):
                refill()
                fresh.append(ev(call))
            reread = sorted(ev(call, 10) for _ in range(3))[1]
            algo = 9 * n * 4
            row.setdefault(f"mode{mode}/fresh_GB_s", []).append(round(algo / sorted(fresh)[4] / 1e6, 1))
            row.setdefault(f"mode{mode}/reread_GB_s", []).append(round(algo / reread / 1e6, 1))
    L.msx_tune_tree(0, 0)
    res[str(mib)] = {k: sorted(v)[1] for k, v in row.items()}
    res[str(mib)]["bit_identical"] = bool(torch.equal(outs[4].view(torch.int32), outs[15].view(torch.int32)))
    print(json.dumps({mib: res[str(mib)]}), file=sys.stderr, flush=True)
print(json.dumps(res), flush=True)
