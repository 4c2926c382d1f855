"""Local copy probe (measurement only): 256 MiB device-to-device copies with
the HBM probe's copy kernel (msx_probe_hbm mode 2), the engine's segment-copy
kernel k_copy_segs (mode 4, the scatter/collect/allgather copies) and
hipMemcpyAsync (mode 5), and the copy kernel forced into each geometry
(modes 8 / 9: XCD-contiguous 4-KiB tiles / one-wave dispatch order), between cached (hipMalloc) and uncached (the engine
windows' memory type) allocations.  GB/s counts read + write bytes."""
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "microsoft-mpi_amd"))
import torch  # noqa: E402

import msx  # noqa: E402

L = msx.init(errors_return=True)
stream = torch.cuda.Stream()
sp = ctypes.c_void_p(stream.cuda_stream)
NB = int(os.environ.get("COPY_BYTES", str(256 << 20)))


def alloc(nbytes, uncached):
    q = ctypes.c_void_p()
    assert L.msx_probe_alloc(nbytes, uncached, ctypes.byref(q)) == 0, msx.last_error()
    return q.value


def timed(fn, reps=20):
    ts = []
    for _ in range(3):
        fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            assert fn() == 0, msx.last_error()
        e1.record(stream)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / reps)
    return sorted(ts)[1]


out = {}
for src_uc, dst_uc in ((0, 0), (1, 0), (0, 1)):
    a, b = alloc(NB, src_uc), alloc(NB, dst_uc)
    for mode, name in ((2, "probe_copy"), (4, "k_copy_segs"), (5, "hipMemcpyAsync"), (8, "forced_xcd_tiles"),
                       (9, "forced_dram_dispatch")):
        ms = timed(lambda: L.msx_probe_hbm(mode, a, b, NB, sp))
        out[f"{'uc' if src_uc else 'c'}->{'uc' if dst_uc else 'c'}/{name}"] = {
            "us": round(ms * 1e3, 1), "GB_s": round(2 * NB / ms / 1e6, 1)}
    L.msx_probe_free(a)
    L.msx_probe_free(b)
print(json.dumps(out), flush=True)
