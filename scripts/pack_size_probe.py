"""Pack / unpack geometry by size (measurement only): the grid-stride form
(msx_tune_pack 1) against the one-wave tile form (2) for the bench's two
granule-mapped layouts (a vector of 16-B blocks at a 32-B stride,
MPI_DOUBLE_INT records) over typed buffers of PACK_MIB (default 256, 1024,
2048) MiB, interleaved rounds, HIP events.  Both forms must produce identical
bytes.  Prints one JSON line."""
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
HBM = 8000.0


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
sizes = [int(x) for x in os.environ.get("PACK_MIB", "256,1024,2048").split(",")]
for mib in sizes:
    nf = mib << 18
    typed = torch.randn(nf, device=dev)
    vt = ctypes.c_int()
    assert L.MPI_Type_vector(nf // 8, 4, 8, C.MPI_FLOAT, ctypes.byref(vt)) == 0
    assert L.MPI_Type_commit(ctypes.byref(vt)) == 0
    layouts = [("vector_16B_blocks_stride32B", vt.value, 1, nf * 2), ("double_int_records_12of16B",
               C.MPI_DOUBLE_INT, nf // 4, nf * 3)]
    for name, t, count, nb in layouts:
        packed = torch.empty(nb, dtype=torch.uint8, device=dev)
        ref = None
        for rnd in range(2):
            for mode in (1, 2):
                assert L.msx_tune_pack(mode) == 0
                torch.cuda.synchronize()
                assert L.msx_pack_dev(typed.data_ptr(), count, t, packed.data_ptr(), sp) == 0, msx.last_error()
                torch.cuda.synchronize()
                if ref is None:
                    ref = packed.clone()
                elif not torch.equal(packed, ref):
                    out[f"{mib}/{name}/mode{mode}/mismatch"] = True
                for label, fn, a, b in (("pack", L.msx_pack_dev, typed, packed),
                                        ("unpack", L.msx_unpack_dev, packed, typed)):
                    ms = timed(lambda: fn(a.data_ptr(), count, t, b.data_ptr(), sp))
                    key = f"{mib}/{name}/{label}/{'grid_stride' if mode == 1 else 'tile'}"
                    out.setdefault(key, []).append(round(ms * 1e3, 1))
        del packed, ref
    L.MPI_Type_free(ctypes.byref(vt))
    del typed
    torch.cuda.empty_cache()
assert L.msx_tune_pack(0) == 0
print(json.dumps(out), flush=True)
