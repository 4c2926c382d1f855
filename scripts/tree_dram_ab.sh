#!/bin/bash
# Tree geometry in the DRAM regime (sources far above the 256 MiB Infinity
# Cache): modes 0 (default = 12 there), 14 (dispatch order), 15/16 (64-lane
# workgroups, dispatch order / XCD-contiguous), per-source 64 and 128 MiB,
# two interleaved rounds.  usage: scripts/tree_dram_ab.sh OUTDIR
cd "$(dirname "$0")/.." || exit 2
OUT=${1:-gpurun_out/tree_dram}
mkdir -p "$OUT"
set -o pipefail
for round in 1 2; do
  for mib in 64 128; do
    TREE_MIB=$mib TREE_MODES=0,12,14,15,16 TREE_CAPS=0 TREE_ORDERS=2147483647 timeout -k 10 180 python scripts/tree_probe.py > "$OUT/tree_${mib}_r${round}.json" 2> "$OUT/tree_${mib}_r${round}.err" || exit 3
    echo "round $round ${mib} MiB done"
  done
done
