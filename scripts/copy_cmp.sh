#!/bin/bash
# Engine copy settings on the shared GPU: allreduce with 2 ranks at 64 MiB
# (two-step) and 1 GiB (host-barrier chunks, collect overlapping the next
# scatter), for the blit (MSX_KERNEL_COPY_MIN=0) and the copy kernel at
# several grid caps (MSX_COPY_GRID_CAP); plus the local copy probe per cap.
cd "$(dirname "$0")/.." || exit 2
OUT=gpurun_out/copy_cmp
mkdir -p "$OUT"
for cap in 1024 4096 16384 0; do
  MSX_COPY_GRID_CAP=$cap timeout -k 5 60 python scripts/copy_probe.py | sed "s/^/cap=$cap /" || exit 1
done
for sz in 67108864 1073741824; do
  for rep in 1 2; do
    for cfg in "0 0" "1048576 0" "1048576 1024" "1048576 4096" "1048576 16384"; do
      set -- $cfg
      MSX_KERNEL_COPY_MIN=$1 MSX_COPY_GRID_CAP=$2 bash scripts/allreduce_probe.sh 2 $sz 10 "$OUT/s${sz}_$1_$2_$rep" allreduce \
        | grep "rank 0" | sed "s/^/kcopy=$1 cap=$2 /" || exit 1
    done
  done
done
