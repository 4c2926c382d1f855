#!/bin/bash
# Does the uncached-free effect (scripts/va_reuse_probe.py) cross processes?
# Process A uses and frees uncached buffers (and exits, which frees the rest);
# process B then runs the probe's checks with no uncached memory of its own
# (the "plain_full" control variant only).  Repeated 4 times.  Output under $1.
cd "$(dirname "$0")/.." || exit 2
OUT=${1:-gpurun_out/xproc}
mkdir -p "$OUT"
for i in 1 2 3 4; do
  timeout -k 10 120 python - > "$OUT/a_$i.log" 2>&1 <<'PY' || exit $?
import ctypes, os, sys, torch
sys.path.insert(0, os.path.join(os.getcwd(), "microsoft-mpi_amd"))
from msx import probe
P = probe.lib()
sp = ctypes.c_void_p(0)
scratch = torch.empty(8 << 18, dtype=torch.int32, device="cuda")
for rep in range(8):
    for mib in (1, 2, 4, 8):
        u = ctypes.c_void_p()
        assert P.msxp_alloc(mib << 20, 1, ctypes.byref(u)) == 0
        assert P.msxp_hbm(probe.WRITE1, None, u, mib << 20, sp) == 0
        assert P.msxp_hbm(probe.COPY, u, scratch.data_ptr(), mib << 20, sp) == 0
        torch.cuda.synchronize()
        if rep < 7:
            assert P.msxp_free(u) == 0      # the last round stays allocated until exit
print("A done")
PY
  timeout -k 10 200 python scripts/va_reuse_probe.py 32 plain > "$OUT/b_$i.log" 2>&1 || exit $?
done
