#!/bin/bash
# Round-4 evidence on one GPU box: N=1 bench, its rocprofv3 kernel statistics,
# two PMC passes (FETCH_SIZE, WRITE_SIZE; one counter group each), smoke.
# Stops at the first failing step.
cd "$(dirname "$0")/.." || exit 2
OUT=${OUT:-gpurun_out/r04}
mkdir -p "$OUT"
export TMPDIR=/tmp
set -o pipefail
# progress marker every 30 s (each step below has its own time limit)
( while sleep 30; do date +%T >> "$OUT/heartbeat"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 400 python bench.py > "$OUT/bench_n1.json" 2> "$OUT/bench_n1.err" || exit 3
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$OUT/prof_trace" -o trace --output-format csv -- python bench.py > "$OUT/bench_under_rocprof.json" 2> "$OUT/rocprof_trace.err" || exit 4
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/prof_pmc" -o pmc_fetch --output-format csv -- python bench.py --steps 10 --warmup 2 --cpu-seconds 0.5 --no-host-path --no-collectives > "$OUT/pmc_fetch.log" 2>&1 || exit 5
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/prof_pmc" -o pmc_write --output-format csv -- python bench.py --steps 10 --warmup 2 --cpu-seconds 0.5 --no-host-path --no-collectives > "$OUT/pmc_write.log" 2>&1 || exit 6
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit 7
# PMC traffic of the fold trees (tree_fixed MASKED) against their algorithmic bytes
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d "$OUT/prof_fold" -o fold_fetch --output-format csv -- python scripts/tree_fold_probe.py 128 > "$OUT/fold_pmc_fetch.log" 2>&1 || exit 9
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d "$OUT/prof_fold" -o fold_write --output-format csv -- python scripts/tree_fold_probe.py 128 > "$OUT/fold_pmc_write.log" 2>&1 || exit 10
timeout -k 10 500 python bench.py --gpus 2 --steps 20 --warmup 5 --no-per-op > "$OUT/bench_n2_shared_gpu.json" 2> "$OUT/bench_n2.err" || exit 8
echo done
