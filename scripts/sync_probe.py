"""Does a synchronisation return before the work it waits for has finished?
A one-workgroup kernel (probe library msxp_spin_mark) waits a few ms, then
writes a value to page-locked host memory; right after hipStreamSynchronize /
hipDeviceSynchronize / hipEventSynchronize / torch.cuda.synchronize returns,
the host reads that word.  Checked before any uncached allocation, after
uncached allocations were used and freed (what a communicator free does to its
engine window), and after plain ones were (the control); on a side stream and
on the null stream.  One JSON line: early returns per phase and sync kind.
usage: python scripts/sync_probe.py [reps]    (GPU only)"""
import ctypes
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "microsoft-mpi_amd"))
from msx import probe  # noqa: E402

P = probe.lib()
hip = ctypes.CDLL("libamdhip64.so")
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 16
dev = torch.device("cuda:0")
torch.cuda.init()
side = torch.cuda.Stream(dev)
h, d = ctypes.c_void_p(), ctypes.c_void_p()
assert hip.hipHostMalloc(ctypes.byref(h), ctypes.c_size_t(64), 0) == 0
assert hip.hipHostGetDevicePointer(ctypes.byref(d), h, 0) == 0
flag = ctypes.cast(h, ctypes.POINTER(ctypes.c_uint32))
flag[0] = 0
scratch = torch.empty(8 << 18, dtype=torch.int32, device=dev)
TICKS = 300_000     # 3 ms at 100 MHz
val = [0]


def run(kind, stream):
    sp = ctypes.c_void_p(stream.cuda_stream if stream is not None else 0)
    early = 0
    for _ in range(reps):
        val[0] += 1
        v = val[0]
        assert P.msxp_spin_mark(TICKS, d, v, sp) == 0
        if kind == "stream":
            rc = hip.hipStreamSynchronize(sp)
        elif kind == "device":
            rc = hip.hipDeviceSynchronize()
        elif kind == "torch":
            torch.cuda.synchronize()
            rc = 0
        else:
            ev = ctypes.c_void_p()
            assert hip.hipEventCreate(ctypes.byref(ev)) == 0
            assert hip.hipEventRecord(ev, sp) == 0
            rc = hip.hipEventSynchronize(ev)
            hip.hipEventDestroy(ev)
        assert rc == 0, (kind, rc)
        if flag[0] != v:
            early += 1
            t0 = time.time()
            while flag[0] != v and time.time() - t0 < 5:
                pass
            assert flag[0] == v, "kernel never finished"
    return early


def phase():
    out = {}
    for sname, st in (("side", side), ("null", None)):
        for kind in ("stream", "device", "torch", "event"):
            out[f"{sname}/{kind}"] = run(kind, st)
    return out


def churn(uncached):
    sp = ctypes.c_void_p(0)
    for mib in (1, 2, 4, 8):
        u = ctypes.c_void_p()
        assert P.msxp_alloc(mib << 20, uncached, ctypes.byref(u)) == 0
        assert P.msxp_hbm(probe.WRITE1, None, u, mib << 20, sp) == 0
        assert P.msxp_hbm(probe.COPY, u, scratch.data_ptr(), mib << 20, sp) == 0
        assert hip.hipDeviceSynchronize() == 0
        assert P.msxp_free(u) == 0


res = {"reps": reps, "spin_ms": TICKS / 1e5}
res["baseline"] = phase()
churn(0)
res["after_plain_free"] = phase()
churn(1)
res["after_uncached_free"] = phase()
res["after_uncached_free_again"] = phase()
print(json.dumps(res))
