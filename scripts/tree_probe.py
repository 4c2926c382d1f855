"""Tree-combine tuning probe (measurement only): p = 8 fp32 SUM sources of
32 MiB in the engine window's IN layout (sub-slots 32 MiB + 68 KiB apart),
in cached (hipMalloc) and uncached (the windows' memory type) allocations,
timed with HIP events for every msx_tune_tree mode and grid cap; plus the
2-operand combine over the same two memory types.  Prints one JSON line."""
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
P, M = 8, int(os.environ.get("TREE_MIB", "32")) << 18   # 8 sources of TREE_MIB MiB of fp32 (default 32)
skew = int(os.environ.get("TREE_SKEW_KB", "68")) << 10
SLOT = M * 4 + skew
HBM = 8000.0


def alloc(nbytes, uncached):
    q = ctypes.c_void_p()
    assert L.msx_probe_alloc(nbytes, uncached, ctypes.byref(q)) == 0, msx.last_error()
    return q.value


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


out = {}
modes = [(0, "default"), (8, "generic"), (1, "generic_upfront"), (2, "generic_upfront_nt"), (3, "generic_nt"),
         (4, "fixed_u1"), (5, "fixed_u2"),
         (6, "fixed_u4"), (7, "fixed_u2_nt"), (9, "fixed_u1_order"), (10, "fixed_u1_b512"),
         (11, "fixed_u1_b1024"), (12, "fixed_u1_nt"), (13, "fixed_u4_nt"), (14, "fixed_u1_nt_order"),
         (15, "fixed_u1_nt_b64_dispatch"), (16, "fixed_u1_nt_b64_xcd"), (17, "generic_nt_b64_dispatch")]
if os.environ.get("TREE_MODES"):
    keep = {int(m) for m in os.environ["TREE_MODES"].split(",")}
    modes = [(m, n) for m, n in modes if m in keep]
caps = [int(c) for c in os.environ.get("TREE_CAPS", "0,1024,2048,4096,8192,65536").split(",")]
# mode 9 reads its "cap" as the tile order (TreeArgs::xg): 0 XCD-contiguous,
# G > 0 runs of G tiles per XCD, 2147483647 dispatch order
orders = [int(c) for c in os.environ.get("TREE_ORDERS", "0,1,4,16,64,256,1024,2147483647").split(",")]
for uncached in (0, 1):
    base = alloc(P * SLOT, uncached)
    dst = alloc(M * 4, uncached)
    t = torch.empty(M, dtype=torch.float32, device=dev)
    t.uniform_(-1, 1)
    torch.cuda.synchronize()
    for r in range(P):   # distinct data per source (a p = 1 tree is a device copy)
        t.uniform_(-1, 1)
        torch.cuda.synchronize()
        L.msx_reduce_tree_dev((ctypes.c_void_p * 1)(t.data_ptr()), 1, base + r * SLOT, M, C.MPI_FLOAT, C.MPI_SUM, sp)
        torch.cuda.synchronize()
    srcs = (ctypes.c_void_p * P)(*[base + r * SLOT for r in range(P)])
    # the reference tree ((s0+s1)+(s2+s3))+((s4+s5)+(s6+s7)) with torch's fp32 adds
    xs = []
    for r in range(P):
        x = torch.empty(M, dtype=torch.float32, device=dev)
        L.msx_reduce_tree_dev((ctypes.c_void_p * 1)(base + r * SLOT), 1, x.data_ptr(), M, C.MPI_FLOAT, C.MPI_SUM, sp)
        xs.append(x)
    torch.cuda.synchronize()
    while len(xs) > 1:
        xs = [xs[2 * k] + xs[2 * k + 1] for k in range(len(xs) // 2)]
    ref = xs[0]
    del xs
    for mode, name in modes:
        for cap in (orders if mode in (9, 14) else caps if mode in (0, 1, 4, 5, 6, 7, 8) else [0]):
            L.msx_tune_tree(mode, cap)
            ms = timed(lambda: L.msx_reduce_tree_dev(srcs, P, dst, M, C.MPI_FLOAT, C.MPI_SUM, sp))
            gbs = (P + 1) * M * 4 / ms / 1e6
            out[f"{'uc' if uncached else 'cached'}/{name}/cap{cap}"] = {"us": round(ms * 1e3, 1),
                                                                        "GB_s": round(gbs, 1),
                                                                        "frac": round(gbs / HBM, 4)}
            # every mode evaluates the same tree: results must agree bit for bit
            got = torch.empty(M, dtype=torch.float32, device=dev)
            L.msx_reduce_tree_dev((ctypes.c_void_p * 1)(dst), 1, got.data_ptr(), M, C.MPI_FLOAT, C.MPI_SUM, sp)
            torch.cuda.synchronize()
            if not torch.equal(got, ref):
                out[f"{'uc' if uncached else 'cached'}/{name}/cap{cap}"]["mismatch"] = True
    L.msx_tune_tree(0, 0)
    # the 2-operand combine over this memory type (sources 0 and 1 -> in, inout)
    a, b = base, base + SLOT
    ms = timed(lambda: L.msx_reduce_local_dev(a, b, M, C.MPI_FLOAT, C.MPI_SUM, sp), reps=20)
    out[f"{'uc' if uncached else 'cached'}/combine2"] = {"us": round(ms * 1e3, 1),
                                                          "GB_s": round(3 * M * 4 / ms / 1e6, 1)}
    L.msx_probe_free(base)
    L.msx_probe_free(dst)
print(json.dumps(out), flush=True)
