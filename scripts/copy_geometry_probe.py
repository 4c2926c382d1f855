"""Local copy geometry by size (measurement only): k_copy_segs' XCD-contiguous
tiles (msx_probe_hbm mode 8) against k_copy_dram's one-wave workgroups in
dispatch order (mode 9), back to back and with the Infinity Cache flushed
before each launch (a 1 GiB read + write pass over other data).  HIP events,
median of 3 rounds of 10 launches (back to back) or of 12 single launches
(cold).  Prints one JSON line {size_MiB: {geometry/warm|cold: GB/s}}."""
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "microsoft-mpi_amd"))
import torch  # noqa: E402

import msx  # noqa: E402

L = msx.init(errors_return=True)
dev = torch.device("cuda:0")
stream = torch.cuda.Stream()
sp = ctypes.c_void_p(stream.cuda_stream)
flush = torch.empty(1 << 30, dtype=torch.uint8, device=dev)


def ev_ms(fn, k):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(k):
        fn()
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / k


out = {}
for mib in [int(x) for x in os.environ.get("SIZES", "16,32,64,128,256").split(",")]:
    nb = mib << 20
    a = torch.randint(0, 256, (nb,), dtype=torch.uint8, device=dev)
    b = torch.zeros(nb, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    row = {}
    for _ in range(int(os.environ.get("ROUNDS", "3"))):
        for mode, name in ((8, "tiles"), (9, "dispatch_order")):
            fn = lambda: L.msx_probe_hbm(mode, a.data_ptr(), b.data_ptr(), nb, sp)
            fn()
            torch.cuda.synchronize()
            assert torch.equal(a, b), (mib, name)
            warm = sorted(ev_ms(fn, 10) for _ in range(3))[1]
            cold = []
            for _ in range(12):
                L.msx_probe_hbm(3, flush.data_ptr(), flush.data_ptr(), flush.numel(), sp)
                L.msx_probe_hbm(1, flush.data_ptr(), flush.data_ptr(), flush.numel(), sp)
                cold.append(ev_ms(fn, 1))
            cms = sorted(cold)[6]
            row.setdefault(name + "/warm", []).append(round(2 * nb / warm / 1e6, 1))
            row.setdefault(name + "/cold", []).append(round(2 * nb / cms / 1e6, 1))
            b.zero_()
            torch.cuda.synchronize()      # the library's stream does not order after torch's
    out[str(mib)] = {k: sorted(v)[len(v) // 2] for k, v in row.items()}
    print(json.dumps({mib: out[str(mib)]}), file=sys.stderr, flush=True)
    del a, b
    torch.cuda.empty_cache()
print(json.dumps(out), flush=True)
