"""fp32 SUM combine: the product kernel against the probe library's launch
geometries of the same body (tile orders, workgroup sizes), back to back and
with the Infinity Cache flushed before each launch, interleaved rounds in one
process.  Every variant is checked bit-exact against torch's fp32 add first.
Prints one JSON line {MiB: {name: {"warm_us", "cold_us", "warm_frac", "cold_frac"}}}.
usage: python scripts/combine_geometry_probe.py [MiB,...] [rounds]    (GPU only)"""
import ctypes
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "microsoft-mpi_amd"))
import msx  # noqa: E402
from msx import probe  # noqa: E402

L = msx.init(errors_return=True)
C = msx.C
P = probe.lib()
sizes = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "256").split(",")]
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
dev = torch.device("cuda:0")
stream = torch.cuda.Stream(dev)
torch.cuda.set_stream(stream)
sp = ctypes.c_void_p(stream.cuda_stream)
flush = torch.empty(1 << 30, dtype=torch.uint8, device=dev)


def flush_cache():
    P.msxp_hbm(probe.READ1, flush.data_ptr(), flush.data_ptr(), flush.numel(), sp)
    P.msxp_hbm(probe.WRITE1, flush.data_ptr(), flush.data_ptr(), flush.numel(), sp)


out = {}
for mib in sizes:
    n = (mib << 20) // 4
    a = torch.rand(n, device=dev) * 2 - 1
    b = torch.rand(n, device=dev) * 2 - 1
    runs = {"product": lambda: L.msx_reduce_local_dev(a.data_ptr(), b.data_ptr(), n, C.MPI_FLOAT, C.MPI_SUM, sp)}
    for name, v in probe.variants().items():
        runs[name] = (lambda v=v: P.msxp_variant_run(v, a.data_ptr(), b.data_ptr(), n, sp))
    # parity of every variant on this size (one IEEE add per element)
    for name in runs:
        c = b.clone()
        want = c + a
        torch.cuda.synchronize()
        rc = (L.msx_reduce_local_dev(a.data_ptr(), c.data_ptr(), n, C.MPI_FLOAT, C.MPI_SUM, sp) if name == "product"
              else P.msxp_variant_run(probe.variants()[name], a.data_ptr(), c.data_ptr(), n, sp))
        torch.cuda.synchronize()
        assert rc == 0 and torch.equal(c.view(torch.int32), want.view(torch.int32)), name
        del c, want
    warm = {k: [] for k in runs}
    cold = {k: [] for k in runs}
    for _ in range(rounds):
        for name, fn in runs.items():
            for _ in range(3):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(10):
                fn()
            e1.record(stream)
            torch.cuda.synchronize()
            warm[name].append(e0.elapsed_time(e1) / 10)
            ts = []
            for _ in range(5):
                flush_cache()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                fn()
                e1.record(stream)
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            cold[name].append(sorted(ts)[2])
    res = {}
    for name in runs:
        w = sorted(warm[name])[len(warm[name]) // 2]
        c = sorted(cold[name])[len(cold[name]) // 2]
        res[name] = {"warm_us": round(w * 1e3, 1), "cold_us": round(c * 1e3, 1),
                     "warm_frac": round(12 * n / w / 1e6 / 8000, 4), "cold_frac": round(12 * n / c / 1e6 / 8000, 4)}
        print(f"{mib} MiB {name}: warm {w * 1e3:.1f} us cold {c * 1e3:.1f} us", file=sys.stderr)
    # the local copy (1R1W) in the same orders: k_copy_segs' 256-lane tiles,
    # k_copy_dram's dispatch order, XCD runs of 128 tiles
    copies = {"copy_tiles256": probe.COPY, "copy_dispatch": probe.COPY_DISPATCH_ORDER,
              "copy_xcd_runs128": probe.COPY_XCD_RUNS}
    cw, cc = {k: [] for k in copies}, {k: [] for k in copies}
    for _ in range(rounds):
        for name, mode in copies.items():
            fn = lambda: P.msxp_hbm(mode, a.data_ptr(), b.data_ptr(), n * 4, sp)
            for _ in range(3):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(10):
                fn()
            e1.record(stream)
            torch.cuda.synchronize()
            cw[name].append(e0.elapsed_time(e1) / 10)
            ts = []
            for _ in range(5):
                flush_cache()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                fn()
                e1.record(stream)
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            cc[name].append(sorted(ts)[2])
    for name in copies:
        w, c = sorted(cw[name])[len(cw[name]) // 2], sorted(cc[name])[len(cc[name]) // 2]
        res[name] = {"warm_us": round(w * 1e3, 1), "cold_us": round(c * 1e3, 1),
                     "warm_frac": round(8 * n / w / 1e6 / 8000, 4), "cold_frac": round(8 * n / c / 1e6 / 8000, 4)}
    out[str(mib)] = res
    del a, b
    torch.cuda.empty_cache()
print(json.dumps(out))
