#!/bin/bash
# bench_collectives.py with P ranks sharing GPU 0 (one-GPU box rehearsal of
# the driver's multi-GPU run). Usage: scripts/coll_shared_gpu.sh P OUT.json [scale]
P=${1:-2}; OUT=${2:-gpurun_out/coll.json}; SCALE=${3:-1.0}
PORT=$((20000 + RANDOM % 20000))
pids=()
for ((r = 0; r < P; r++)); do
  MSX_SIZE=$P MSX_RANK=$r MSX_DEVICE=0 MSX_BOOTSTRAP_ADDR=127.0.0.1 MSX_BOOTSTRAP_PORT=$PORT \
  MSX_BOOTSTRAP_TIMEOUT=90 MSX_BENCH_LOG=${OUT%.json}.log \
    timeout -k 10 240 python3 bench_collectives.py "$OUT" "$SCALE" &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait "$p" || rc=$?; done
exit $rc
