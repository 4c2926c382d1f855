#!/usr/bin/env python3
"""Small-call latency breakdown of the device MPI_Reduce_local path (8 B fp32
SUM), without torch: hipMalloc'd operands through ctypes.
  reduce_local   MPI_Reduce_local (2 pointer queries + launch + sync)
  dev_launch     msx_reduce_local_dev + hipStreamSynchronize (no pointer queries)
  ptr_query      hipPointerGetAttributes alone
  memset_sync    hipMemsetAsync(4 B) + hipStreamSynchronize (runtime floor)
Usage: python scripts/latency_probe.py [ITERS]   (env: HIP_* knobs under test;
MSX_PROBE_SPIN=1 sets hipDeviceScheduleSpin before the first HIP call)."""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "microsoft-mpi_amd"))
hip = ctypes.CDLL("libamdhip64.so")
if os.environ.get("MSX_PROBE_SPIN") == "1":
    assert hip.hipSetDeviceFlags(1) == 0          # hipDeviceScheduleSpin
import msx  # noqa: E402

L = msx.init(errors_return=True)
C = msx.C
it = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
a, b = ctypes.c_void_p(), ctypes.c_void_p()
assert hip.hipMalloc(ctypes.byref(a), 64) == 0 and hip.hipMalloc(ctypes.byref(b), 64) == 0
s = ctypes.c_void_p()
assert hip.hipStreamCreate(ctypes.byref(s)) == 0
attr = ctypes.create_string_buffer(256)


def timeit(fn):
    for _ in range(200):
        fn()
    t0 = time.perf_counter()
    for _ in range(it):
        fn()
    return round((time.perf_counter() - t0) / it * 1e6, 2)


res = {
    "reduce_local": timeit(lambda: L.MPI_Reduce_local(a, b, 2, C.MPI_FLOAT, C.MPI_SUM)),
    "dev_launch": timeit(lambda: (L.msx_reduce_local_dev(a, b, 2, C.MPI_FLOAT, C.MPI_SUM, s),
                                  hip.hipStreamSynchronize(s))),
    "ptr_query": timeit(lambda: hip.hipPointerGetAttributes(attr, a)),
    "memset_sync": timeit(lambda: (hip.hipMemsetAsync(a, 0, 4, s), hip.hipStreamSynchronize(s))),
}
res["env"] = {k: v for k, v in os.environ.items() if k.startswith(("HIP_", "MSX_PROBE", "AMD_", "HSA_"))
              and k != "HSA_ENABLE_IPC_MODE_LEGACY"}
print(json.dumps(res), flush=True)
