"""Infinity Cache (MALL, 256 MiB on MI355X) check for the HBM numbers
(measurement only): the k_probe stream mixes and the fp32 SUM combine at
several operand sizes, each re-run 10x back to back like the bench.  A working
set that fits (or nearly fits) the MALL is partly served from it; far above it
the rates are DRAM's.  Prints one JSON line: {size_MiB: {probe: GB/s}}."""
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
dev = torch.device("cuda:0")
stream = torch.cuda.Stream()
sp = ctypes.c_void_p(stream.cuda_stream)


def timed(fn, reps=10):
    ts = []
    for _ in range(3):
        fn()
        fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            fn()
        e1.record(stream)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / reps)
    return sorted(ts)[1]


out = {}
flush = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
for mib in [int(x) for x in os.environ.get("MALL_SIZES", "64,128,256,512,1024,2048").split(",")]:
    nb = mib << 20
    a = torch.empty(nb, dtype=torch.uint8, device=dev)
    b = torch.empty(nb, dtype=torch.uint8, device=dev)
    with torch.cuda.stream(stream):
        a.random_(0, 256)
        b.random_(0, 256)
        af, bf = a.view(torch.float32), b.view(torch.float32)
        af.uniform_(-1, 1)
        bf.uniform_(-1, 1)
    torch.cuda.synchronize()
    row = {}
    for mode, name, streams in ((0, "read2", 2), (3, "read1", 1), (1, "write1", 1), (2, "copy_r1w1", 2)):
        ms = timed(lambda: L.msx_probe_hbm(mode, a.data_ptr(), b.data_ptr(), nb, sp))
        row[name] = round(streams * nb / ms / 1e6, 1)
    n = nb // 4
    ms = timed(lambda: L.msx_reduce_local_dev(a.data_ptr(), b.data_ptr(), n, C.MPI_FLOAT, C.MPI_SUM, sp))
    row["combine_fp32_sum"] = round(3 * nb / ms / 1e6, 1)
    row["combine_us"] = round(ms * 1e3, 1)
    # cold: before each timed launch, stream 1 GiB of other data through the
    # caches (a read + a write pass over `flush`), so the Infinity Cache holds
    # none of the operands; one launch per pair of events
    cold = []
    for _ in range(12):
        L.msx_probe_hbm(3, flush.data_ptr(), flush.data_ptr(), flush.numel(), sp)
        L.msx_probe_hbm(1, flush.data_ptr(), flush.data_ptr(), flush.numel(), sp)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        L.msx_reduce_local_dev(a.data_ptr(), b.data_ptr(), n, C.MPI_FLOAT, C.MPI_SUM, sp)
        e1.record(stream)
        torch.cuda.synchronize()
        cold.append(e0.elapsed_time(e1))
    cms = sorted(cold)[len(cold) // 2]
    row["combine_cold_fp32_sum"] = round(3 * nb / cms / 1e6, 1)
    row["combine_cold_us"] = round(cms * 1e3, 1)
    # warm single launch with the same event bracketing (launch-overhead control)
    warm = []
    for _ in range(12):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        L.msx_reduce_local_dev(a.data_ptr(), b.data_ptr(), n, C.MPI_FLOAT, C.MPI_SUM, sp)
        e1.record(stream)
        torch.cuda.synchronize()
        warm.append(e0.elapsed_time(e1))
    wms = sorted(warm)[len(warm) // 2]
    row["combine_single_warm_us"] = round(wms * 1e3, 1)
    out[str(mib)] = row
    del a, b, af, bf
    torch.cuda.empty_cache()
    print(json.dumps({mib: row}), file=sys.stderr, flush=True)
print(json.dumps(out), flush=True)
