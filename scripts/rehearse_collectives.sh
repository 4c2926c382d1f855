#!/bin/bash
# Rehearse bench_collectives.py (the c3-c5 harness bench.py runs at N > 1) with
# P ranks sharing this box's GPU at a reduced size: validates the P-rank code
# paths and the harness, not xGMI performance.   usage: rehearse_collectives.sh P SCALE
P=${1:-8}; SCALE=${2:-0.05}
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
PORT=$((20000 + RANDOM % 20000))
pids=()
for ((r = 0; r < P; r++)); do
    MSX_SIZE=$P MSX_RANK=$r MSX_DEVICE=0 MSX_BOOTSTRAP_ADDR=127.0.0.1 MSX_BOOTSTRAP_PORT=$PORT \
    MSX_BOOTSTRAP_TIMEOUT=120 MSX_BENCH_LOG=gpurun_out/rehearse_p$P.log \
        timeout -k 10 300 python bench_collectives.py gpurun_out/rehearse_p$P.json "$SCALE" \
        > gpurun_out/rehearse_p${P}_r$r.out 2>&1 &
    pids+=($!)
done
rc=0
for pid in "${pids[@]}"; do wait "$pid" || rc=$?; done
echo "exit $rc"
cat gpurun_out/rehearse_p$P.json
exit $rc
