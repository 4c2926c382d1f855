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
    # the run-parallel kernel (k_dt_runs: 3-D fp32 subarray with 1536-B rows, the
    # bench's shape scaled along the outer dimension): one geometry, timed alone
    if os.environ.get("PACK_SUBARRAY", "1") == "1":
        ia = lambda v: (ctypes.c_int * len(v))(*v)
        d0 = nf // (512 * 512)
        dims, sub, st = (d0, 512, 512), (d0 * 3 // 4, 400, 384), (d0 // 8, 56, 64)
        t3 = ctypes.c_int()
        assert L.MPI_Type_create_subarray(3, ia(dims), ia(sub), ia(st), C.MPI_ORDER_C, C.MPI_FLOAT,
                                          ctypes.byref(t3)) == 0
        assert L.MPI_Type_commit(ctypes.byref(t3)) == 0
        nb = sub[0] * sub[1] * sub[2] * 4
        packed = torch.empty(nb, dtype=torch.uint8, device=dev)
        want = typed.view(*dims)[st[0]:st[0] + sub[0], st[1]:st[1] + sub[1], st[2]:st[2] + sub[2]].contiguous()
        torch.cuda.synchronize()
        assert L.msx_pack_dev(typed.data_ptr(), 1, t3.value, packed.data_ptr(), sp) == 0
        torch.cuda.synchronize()
        out[f"{mib}/subarray3d_rows1536B/correct"] = bool(torch.equal(packed, want.view(-1).view(torch.uint8)))
        for rnd in range(2):
            for mode, mname in ((1, "runs"), (2, "tile")):
                assert L.msx_tune_pack(mode) == 0
                assert L.msx_pack_dev(typed.data_ptr(), 1, t3.value, packed.data_ptr(), sp) == 0
                torch.cuda.synchronize()
                if not torch.equal(packed, want.view(-1).view(torch.uint8)):
                    out[f"{mib}/subarray3d_rows1536B/{mname}/mismatch"] = True
                for label, fn, a, b in (("pack", L.msx_pack_dev, typed, packed),
                                        ("unpack", L.msx_unpack_dev, packed, typed)):
                    ms = timed(lambda: fn(a.data_ptr(), 1, t3.value, b.data_ptr(), sp))
                    out.setdefault(f"{mib}/subarray3d_rows1536B/{label}/{mname}", []).append(
                        {"us": round(ms * 1e3, 1), "frac": round(2 * nb / ms / 1e6 / HBM, 4)})
        assert L.msx_tune_pack(0) == 0
        del packed, want
        L.MPI_Type_free(ctypes.byref(t3))
    L.MPI_Type_free(ctypes.byref(vt))
    del typed
    torch.cuda.empty_cache()
assert L.msx_tune_pack(0) == 0
print(json.dumps(out), flush=True)
