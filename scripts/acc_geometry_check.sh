#!/bin/bash
# Derived-target accumulate geometry: timings (scripts/acc_probe.py) and the
# RMA parity suites with the current default.  usage: scripts/acc_geometry_check.sh OUTDIR
cd "$(dirname "$0")/.." || exit 2
OUT=${1:-gpurun_out/acc_geo}
mkdir -p "$OUT"
set -o pipefail
timeout -k 10 300 python scripts/acc_probe.py > "$OUT/acc.json" 2> "$OUT/acc.err" || { tail -20 "$OUT/acc.err"; exit 3; }
cat "$OUT/acc.json"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_rma.py tests/test_gpu_rma_compact.py tests/test_gpu_rma_passive.py tests/test_gpu_rma_pscw.py tests/test_gpu_dtype_multirank.py > "$OUT/rma_tests.log" 2>&1 || { tail -20 "$OUT/rma_tests.log"; exit 4; }
tail -1 "$OUT/rma_tests.log"
