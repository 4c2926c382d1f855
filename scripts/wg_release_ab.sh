#!/bin/bash
# Interleaved A/B of the per-workgroup agent release before completion counts
# (MSX_WG_RELEASE=1, round-4 default) against store completion only (=0):
# flag-synchronised allreduce on P ranks sharing GPU 0, fp32 SUM.
# Usage: scripts/wg_release_ab.sh OUTDIR
OUT=${1:-gpurun_out/wgrel}
mkdir -p "$OUT"
for round in 1 2; do
  for P in 2 4; do
    for N in 4096 1048576 67108864; do
      for M in 0 1; do
        MSX_WG_RELEASE=$M scripts/allreduce_probe.sh $P $N 50 "$OUT/p${P}_n${N}_m${M}_r${round}" allreduce \
          | sed -n "1s/^/rel=$M p=$P /p" || exit 1
      done
    done
  done
done
