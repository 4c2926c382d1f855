"""The 8-source collective tree (fp32 SUM): the product's call
(msx_reduce_tree_dev; plain loads in 256-lane XCD-contiguous tiles up to 256
MiB of sources, non-temporal loads in one-wave workgroups in dispatch order
above) against the probe library's copy of the non-temporal kernel in other
tile orders.  Timed back to back (warm), with the Infinity Cache flushed before
each launch (cold), and with the cache flushed and then the sources rewritten
by kernels right before the launch (fresh: what a collective's tree meets after
the peers' scatter), interleaved rounds.  Sources sit in one uncached
allocation, Q + 68 KiB apart like the engine window's sub-slots.  Every call is
first checked bit-exact against the tree in torch fp32 over the sources as read
back (mismatches are listed, and the exit status is 1).  Prints one JSON line
{MiB per source: {name: {"warm_us", "cold_us", "fresh_us", ..._frac}}};
algorithmic bytes = 9 x the source size (8 reads + 1 write).
usage: python scripts/tree_geometry_probe.py [MiB,...] [rounds]    (GPU only)"""
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
sizes = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "64,128").split(",")]
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
dev = torch.device("cuda:0")
stream = torch.cuda.Stream(dev)
torch.cuda.set_stream(stream)
sp = ctypes.c_void_p(stream.cuda_stream)
flush = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
SKEW = 68 << 10
ORDERS = {"dispatch(product)": -1, "xcd_tiles": 0, "xg32": 32, "xg128": 128, "xg512": 512}


def flush_cache():
    P.msxp_hbm(probe.READ1, flush.data_ptr(), flush.data_ptr(), flush.numel(), sp)
    P.msxp_hbm(probe.WRITE1, flush.data_ptr(), flush.data_ptr(), flush.numel(), sp)


out = {}
mismatches = []
kept = []
for mib in sizes:
    n = (mib << 20) // 4
    stride = mib * (1 << 20) + SKEW
    base = ctypes.c_void_p()
    assert P.msxp_alloc(8 * stride, 1, ctypes.byref(base)) == 0
    fill = torch.rand(n, device=dev) * 2 - 1
    srcs = [base.value + k * stride for k in range(8)]
    for k, a in enumerate(srcs):
        assert P.msxp_hbm(probe.COPY, fill.data_ptr(), ctypes.c_void_p(a), n * 4, sp) == 0
        fill.mul_(-0.5).add_(0.25)
    arr = (ctypes.c_void_p * 8)(*srcs)
    want = torch.empty(n, device=dev)
    got = torch.empty(n, device=dev)
    torch.cuda.synchronize()
    assert L.msx_reduce_tree_dev(arr, 8, want.data_ptr(), n, C.MPI_FLOAT, C.MPI_SUM, sp) == 0
    runs = {"product": lambda: L.msx_reduce_tree_dev(arr, 8, got.data_ptr(), n, C.MPI_FLOAT, C.MPI_SUM, sp)}
    for name, xg in ORDERS.items():
        runs[name] = (lambda xg=xg: P.msxp_tree8(arr, got.data_ptr(), n, xg, sp))
    torch.cuda.synchronize()
    back = []
    for a in srcs:   # the sources as the kernels see them, and the tree in torch fp32
        t = torch.empty(n, device=dev)
        assert P.msxp_hbm(probe.COPY, ctypes.c_void_p(a), t.data_ptr(), n * 4, sp) == 0
        back.append(t)
    torch.cuda.synchronize()
    ref = ((back[0] + back[1]) + (back[2] + back[3])) + ((back[4] + back[5]) + (back[6] + back[7]))
    stage = torch.stack(back)    # the sources' bytes in plain memory, for the "fresh" rewrites
    del back
    for name, fn in [("first product call", None)] + list(runs.items()):
        if fn is not None:
            got.zero_()
            torch.cuda.synchronize()
            assert fn() == 0, name
            torch.cuda.synchronize()
        res = want if fn is None else got
        bad = res.view(torch.int32) != ref.view(torch.int32)
        if bool(bad.any()):
            idx = bad.nonzero().flatten()
            print(f"MISMATCH {mib} MiB/source {name}: {int(bad.sum())} elements, first {int(idx[0])} "
                  f"last {int(idx[-1])}", file=sys.stderr, flush=True)
            mismatches.append([mib, name, int(bad.sum()), int(idx[0]), int(idx[-1])])
    warm = {k: [] for k in runs}
    cold = {k: [] for k in runs}
    fresh = {k: [] for k in runs}
    for _ in range(rounds):
        for name, fn in runs.items():
            for _ in range(2):
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
            # as in a collective: the Infinity Cache flushed, then the sources
            # written by kernels (uncached stores, as the peers' scatter) right
            # before the tree
            ts = []
            for _ in range(5):
                flush_cache()
                for k, a in enumerate(srcs):
                    P.msxp_hbm(probe.COPY, stage[k].data_ptr(), ctypes.c_void_p(a), n * 4, sp)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                fn()
                e1.record(stream)
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            fresh[name].append(sorted(ts)[2])
    res = {}
    for name in runs:
        w = sorted(warm[name])[len(warm[name]) // 2]
        c = sorted(cold[name])[len(cold[name]) // 2]
        f = sorted(fresh[name])[len(fresh[name]) // 2]
        res[name] = {"warm_us": round(w * 1e3, 1), "cold_us": round(c * 1e3, 1), "fresh_us": round(f * 1e3, 1),
                     "warm_frac": round(9 * n * 4 / w / 1e6 / 8000, 4), "cold_frac": round(9 * n * 4 / c / 1e6 / 8000, 4),
                     "fresh_frac": round(9 * n * 4 / f / 1e6 / 8000, 4)}
        print(f"{mib} MiB/source {name}: warm {w * 1e3:.1f} us cold {c * 1e3:.1f} us "
              f"fresh-written {f * 1e3:.1f} us", file=sys.stderr)
    out[str(mib)] = res
    del fill, want, got, stage
    kept.append(base)      # uncached memory is freed only at the end (uc_pool)
    torch.cuda.empty_cache()
out["mismatches"] = mismatches
for b in kept:
    P.msxp_free(b)
print(json.dumps(out))
sys.exit(1 if mismatches else 0)
