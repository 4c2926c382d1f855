#!/bin/bash
# run scripts/small_coll_probe.py with P ranks sharing this box's GPU
# usage: small_coll_probe.sh P
P=${1:-2}; MB=${2:-128}
cd "$(dirname "$0")/.." || exit 2
PORT=$((20000 + RANDOM % 20000))
pids=()
for ((r = 0; r < P; r++)); do
    MSX_SIZE=$P MSX_RANK=$r MSX_DEVICE=0 MSX_BOOTSTRAP_ADDR=127.0.0.1 MSX_BOOTSTRAP_PORT=$PORT \
    MSX_BOOTSTRAP_TIMEOUT=60 timeout -k 10 200 python scripts/small_coll_probe.py &
    pids+=($!)
done
rc=0
for pid in "${pids[@]}"; do wait "$pid" || rc=$?; done
exit $rc
