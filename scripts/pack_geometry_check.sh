#!/bin/bash
# Pack / unpack geometry by size: timings (scripts/pack_size_probe.py), then
# the datatype parity suites with the tile form forced and at the default.
# usage: scripts/pack_geometry_check.sh OUTDIR
cd "$(dirname "$0")/.." || exit 2
OUT=${1:-gpurun_out/pack_geo}
mkdir -p "$OUT"
set -o pipefail
timeout -k 10 300 python scripts/pack_size_probe.py > "$OUT/pack_size.json" 2> "$OUT/pack_size.err" || { tail -20 "$OUT/pack_size.err"; exit 3; }
echo "pack probe done"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dtype.py tests/test_gpu_dtype_multirank.py tests/test_gpu_rma_compact.py > "$OUT/dtype_tests.log" 2>&1 || { tail -20 "$OUT/dtype_tests.log"; exit 4; }
tail -1 "$OUT/dtype_tests.log"
MSX_PACK_TILE_MIN=0 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dtype_multirank.py tests/test_gpu_rma_compact.py tests/test_gpu_rma.py > "$OUT/dtype_tests_tile_forced.log" 2>&1 || { tail -20 "$OUT/dtype_tests_tile_forced.log"; exit 5; }
tail -1 "$OUT/dtype_tests_tile_forced.log"
