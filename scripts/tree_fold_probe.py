"""Non-power-of-two fold trees at DRAM sizes (measurement only): the p = 6
allreduce leaf tree (P = 4 leaves, leaves 0 and 1 folded pairs: 6 sources)
and the p = 7 binomial tree (P = 8, 7 leaves), fp32 SUM over MIB MiB per
source in uncached device memory (the engine windows' type), timed with HIP
events: the round-4 compile-time-leaf kernel (tree_fixed MASKED, the default
dispatch) against the generic kernel in the same DRAM-regime geometry (tuning
mode 17, the round-3 default for these trees) and as it was before that
(mode 8).  Algorithmic bytes per launch = (sources + 1) x MIB MiB.
Usage: python scripts/tree_fold_probe.py [MIB]  -> one JSON line."""
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
MIB = int(sys.argv[1]) if len(sys.argv) > 1 else 128
n = MIB << 18
stream = torch.cuda.Stream()
sp = ctypes.c_void_p(stream.cuda_stream)
HBM = 8000.0
skew = 68 << 10


def alloc(nbytes):
    q = ctypes.c_void_p()
    assert L.msx_probe_alloc(nbytes, 1, ctypes.byref(q)) == 0, msx.last_error()
    return q.value


slot = n * 4 + skew
base = alloc(8 * slot)
srcs = [base + k * slot for k in range(8)]
out_t = torch.empty(n, device="cuda")
fill = torch.rand(n, device="cuda")
for k in range(8):
    assert L.msx_probe_hbm(4, fill.data_ptr(), ctypes.c_void_p(srcs[k]), n * 4, sp) == 0   # engine copy kernel
torch.cuda.synchronize()

def fold(P, pm):
    # leaf k = (slot 2k, slot 2k+1 when paired); sources numbered in slot order
    ptrs, nsrc = [], 0
    for k in range(P):
        a = srcs[nsrc]; nsrc += 1
        b = srcs[nsrc] if (pm >> k) & 1 else a
        nsrc += (pm >> k) & 1
        ptrs += [a, b]
    return ptrs, nsrc


cases = {}
for name, P, pm in (("p3_fold_P2", 2, 0b1), ("p5_fold_P4", 4, 0b1), ("p6_fold_P4", 4, 0b11), ("p7_fold_P4", 4, 0b111)):
    ptrs, ns = fold(P, pm)
    cases[name] = (P, pm, P, ptrs, ns)
for nl in (5, 6, 7):
    cases[f"p{nl}_binomial_P8"] = (8, 0, nl, [srcs[k // 2] if k % 2 == 0 and k // 2 < nl else srcs[0] for k in range(16)], nl)


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


res = {"mib_per_source": MIB, "memory": "uncached (hipDeviceMallocUncached, the windows' type)",
       "timing": "HIP events around 10 launches, median of 3 rounds"}
outs = {}
for name, (P, pm, nl, ptrs, nsrc) in cases.items():
    arr = (ctypes.c_void_p * len(ptrs))(*ptrs)
    for mode, label in ((0, "fixed_masked_default"), (17, "generic_dram_geometry_r03"), (8, "generic_plain")):
        assert L.msx_tune_tree(mode, 0) == 0
        call = lambda: L.msx_reduce_tree_spec_dev(arr, P, pm, nl, 0, out_t.data_ptr(), n, C.MPI_FLOAT, C.MPI_SUM, sp)
        assert call() == 0, msx.last_error()
        torch.cuda.synchronize()
        outs[(name, mode)] = out_t.clone()
        ms = timed(call)
        algo = (nsrc + 1) * n * 4
        gbs = algo / ms / 1e6
        res[f"{name}/{label}"] = {"us": round(ms * 1e3, 1), "GB_s": round(gbs, 1), "frac": round(gbs / HBM, 4),
                                  "bytes_per_launch": algo}
    L.msx_tune_tree(0, 0)
    res[f"{name}/bit_identical_across_kernels"] = all(
        torch.equal(outs[(name, 0)].view(torch.int32), outs[(name, m)].view(torch.int32)) for m in (17, 8))
print(json.dumps(res), flush=True)
