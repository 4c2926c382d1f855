#!/bin/bash
# DRAM-regime geometries of the tree (NT sources) and the local copy:
# timings (copy probe at 512 MiB / 1 GiB, tree A/B at 64 / 128 MiB per
# source) and the parity suites with both forced on for every launch.
# usage: scripts/dram_geometry_check.sh OUTDIR
cd "$(dirname "$0")/.." || exit 2
OUT=${1:-gpurun_out/dram_geo}
mkdir -p "$OUT"
set -o pipefail
for mib in 512 1024; do
  COPY_BYTES=$((mib << 20)) timeout -k 10 120 python scripts/copy_probe.py > "$OUT/copy_${mib}.json" 2> "$OUT/copy_${mib}.err" || exit 3
done
echo "copy probes done"
for mib in 64 128; do
  TREE_MIB=$mib TREE_MODES=0,12,15 TREE_CAPS=0 timeout -k 10 180 python scripts/tree_probe.py > "$OUT/tree_${mib}.json" 2> "$OUT/tree_${mib}.err" || exit 4
done
echo "tree probes done"
export MSX_TREE_NT_MIN=0 MSX_COPY_DRAM_MIN=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_gpu_local.py -k "tree or copy" > "$OUT/forced_local.log" 2>&1 || { tail -20 "$OUT/forced_local.log"; exit 5; }
tail -1 "$OUT/forced_local.log"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_multirank.py tests/test_gpu_nbc.py > "$OUT/forced_multirank.log" 2>&1 || { tail -20 "$OUT/forced_multirank.log"; exit 6; }
tail -1 "$OUT/forced_multirank.log"
unset MSX_TREE_NT_MIN MSX_COPY_DRAM_MIN
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 || { tail -20 "$OUT/gpu_tests.log"; exit 7; }
tail -1 "$OUT/gpu_tests.log"
