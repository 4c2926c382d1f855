#!/bin/bash
# Every size-switched geometry forced on for every launch (DRAM-regime combine,
# non-temporal one-wave trees, k_copy_dram for local copies >= 1 MiB, the pack
# and accumulate tile forms), through the whole -m gpu suite.
cd "$(dirname "$0")/.." || exit 2
OUT=${1:-gpurun_out/stress_dram}
mkdir -p "$OUT"
set -o pipefail
export MSX_COMBINE_DRAM_MIN=0 MSX_TREE_NT_MIN=0 MSX_COPY_DRAM_MIN=0 MSX_PACK_TILE_MIN=0 MSX_ACC_TILE_MIN=0
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests_forced.log" 2>&1 || { tail -30 "$OUT/gpu_tests_forced.log"; exit 3; }
tail -1 "$OUT/gpu_tests_forced.log"
