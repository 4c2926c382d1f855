#!/bin/bash
# A/B of the two-step collectives with plain (MSX_WT_STORES=0) vs write-through
# (default) remote stores: p ranks sharing GPU 0, fp32 SUM, interleaved rounds.
# Usage: scripts/wt_cmp.sh [ROUNDS]   (output: gpurun_out/wt_cmp.log)
cd "$(dirname "$0")/.." || exit 2
OUT=gpurun_out/wt_cmp
mkdir -p "$OUT"
LOG=gpurun_out/wt_cmp.log
: > "$LOG"
R=${1:-2}
for ((i = 0; i < R; i++)); do
  for P in 2 4; do
    for KIND in allreduce rsb reduce; do
      for N in 1048576 67108864; do
        for WT in 0 1; do
          echo "round $i p $P $KIND $N wt $WT" >> "$LOG"
          MSX_WT_STORES=$WT timeout -k 10 200 bash scripts/allreduce_probe.sh "$P" "$N" 50 "$OUT/x" "$KIND" >> "$LOG" 2>&1 || { echo "probe rc=$?"; exit 1; }
        done
      done
    done
  done
done
echo done >> "$LOG"
