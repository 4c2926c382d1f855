#!/bin/bash
# One GPU-box check of the current tree: smoke, the whole -m gpu suite, then a
# 2-rank shared-GPU bench (collectives c3-c5 on the IPC plane; chunks_per_call
# shows the window layout).  Stops at the first failing step.
# usage: scripts/session_check.sh OUTDIR
cd "$(dirname "$0")/.." || exit 2
OUT=${1:-gpurun_out/check}
mkdir -p "$OUT"
set -o pipefail
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "smoke rc=$?"; tail -20 "$OUT/smoke.log"; exit 3; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 || { echo "tests rc=$?"; tail -30 "$OUT/gpu_tests.log"; exit 4; }
tail -1 "$OUT/gpu_tests.log"
timeout -k 10 400 python bench.py --gpus 2 --steps 5 --warmup 2 --no-host-path > "$OUT/bench_n2.json" 2> "$OUT/bench_n2.err" || { echo "bench n2 rc=$?"; tail -20 "$OUT/bench_n2.err"; exit 5; }
python - "$OUT/bench_n2.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
c = d["collectives"]
print(json.dumps(d["collectives_summary"]))
for k in ("c3_allreduce_sum_f32", "c4_reduce_scatter_max_f64", "c5_iallreduce_band_u64"):
    v = c.get(k, {})
    print(k, {x: v.get(x) for x in ("seconds", "t_comm_s", "busbw_GB_s", "chunks_per_call", "correct")})
PY
