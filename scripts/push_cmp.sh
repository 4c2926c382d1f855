#!/bin/bash
# Two-step push geometry (k_push_wait): the earlier default (4 granules per
# lane, <= 2048 workgroups) vs one granule per lane with up to 16384
# workgroups; allreduce / reduce_scatter_block with P ranks sharing GPU 0.
cd "$(dirname "$0")/.." || exit 2
OUT=gpurun_out/push_cmp
mkdir -p "$OUT"
for P in 2 4; do
  for sz in 4194304 16777216 67108864; do
    for kind in allreduce rsb; do
      for cfg in "1024 2048" "256 16384"; do
        set -- $cfg
        MSX_PUSH_VECS=$1 MSX_PUSH_GRID_CAP=$2 bash scripts/allreduce_probe.sh $P $sz 20 "$OUT/p${P}_${sz}_${kind}_$1" $kind \
          | grep "rank 0" | sed "s/^/p=$P vecs=$1 cap=$2 /" || exit 1
      done
    done
  done
done
