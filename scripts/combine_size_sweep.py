"""fp32 SUM combine tuning variants (msx_tune_set) at several operand sizes
(measurement only): the bench's 256 MiB, where the 256 MiB Infinity Cache
still helps, and sizes far above it, where the rate is DRAM's
(scripts/mall_probe.py).  HIP events, median of 3 rounds of 10 launches.
Every variant's result is checked against torch's fp32 add.  Prints one JSON
line {size_MiB: {variant[/capN]: GB/s}}."""
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
L.msx_tune_variant_name.restype = ctypes.c_char_p
dev = torch.device("cuda:0")
stream = torch.cuda.Stream()
sp = ctypes.c_void_p(stream.cuda_stream)
nv = L.msx_tune_variant_count()
names = [L.msx_tune_variant_name(v).decode() for v in range(nv)]
sel = os.environ.get("SWEEP_VARIANTS")
variants = [int(v) for v in sel.split(",")] if sel else list(range(nv))
caps = [int(c) for c in os.environ.get("SWEEP_CAPS", "0").split(",")]


def timed(fn, reps=10):
    ts = []
    for _ in range(3):
        fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            fn()
        e1.record(stream)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / reps)
    return sorted(ts)[1]


COLD = os.environ.get("SWEEP_COLD") == "1"
flush = torch.empty(1 << 30, dtype=torch.uint8, device=dev) if COLD else None


def timed_cold(fn, reps=12):
    """Each launch alone after a 1 GiB read + write pass over other data
    (Infinity Cache cold); median."""
    ts = []
    for _ in range(reps):
        L.msx_probe_hbm(3, flush.data_ptr(), flush.data_ptr(), flush.numel(), sp)
        L.msx_probe_hbm(1, flush.data_ptr(), flush.data_ptr(), flush.numel(), sp)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        fn()
        e1.record(stream)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return sorted(ts)[reps // 2]


out = {}
for mib in [int(x) for x in os.environ.get("SWEEP_SIZES", "256,1024").split(",")]:
    n = (mib << 20) // 4
    a = torch.empty(n, dtype=torch.float32, device=dev).uniform_(-1, 1)
    b0 = torch.empty(n, dtype=torch.float32, device=dev).uniform_(-1, 1)
    b = b0.clone()
    want = b0 + a
    torch.cuda.synchronize()
    row = {}
    runs = {}
    for _ in range(int(os.environ.get("SWEEP_ROUNDS", "1"))):    # interleaved rounds, median
     for v in variants:
        for cap in caps:
            if L.msx_tune_set(v, cap) != 0:
                continue
            b.copy_(b0)
            torch.cuda.synchronize()
            L.msx_reduce_local_dev(a.data_ptr(), b.data_ptr(), n, C.MPI_FLOAT, C.MPI_SUM, sp)
            torch.cuda.synchronize()
            ok = torch.equal(b, want)
            ms = (timed_cold if COLD else timed)(
                lambda: L.msx_reduce_local_dev(a.data_ptr(), b.data_ptr(), n, C.MPI_FLOAT, C.MPI_SUM, sp))
            key = names[v] + (f"/cap{cap}" if cap else "")
            runs.setdefault(key, []).append(round(3 * n * 4 / ms / 1e6, 1) if ok else float("nan"))
    for key, r in runs.items():
        r = sorted(r)
        row[key] = r[len(r) // 2] if r == r else "MISMATCH"
    L.msx_tune_set(0, 0)
    out[str(mib)] = row
    print(json.dumps({mib: row}), file=sys.stderr, flush=True)
    del a, b, b0, want
    torch.cuda.empty_cache()
print(json.dumps(out), flush=True)
