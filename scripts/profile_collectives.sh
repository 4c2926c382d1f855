#!/bin/bash
# rocprofv3 kernel statistics of the c3-c5 collectives harness: P ranks on this
# box's one GPU, each rank under its own `rocprofv3 --kernel-trace --stats`.
# usage: profile_collectives.sh P SCALE   (outputs gpurun_out/prof_coll/rank<r>/)
P=${1:-2}; SCALE=${2:-0.5}
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_coll
PORT=$((20000 + RANDOM % 20000))
pids=()
for ((r = 0; r < P; r++)); do
    MSX_SIZE=$P MSX_RANK=$r MSX_DEVICE=0 MSX_BOOTSTRAP_ADDR=127.0.0.1 MSX_BOOTSTRAP_PORT=$PORT \
    MSX_BOOTSTRAP_TIMEOUT=120 \
        timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_coll/rank$r -o coll \
        --output-format csv -- python bench_collectives.py gpurun_out/prof_coll/coll_p$P.json "$SCALE" \
        > gpurun_out/prof_coll/rank$r.out 2>&1 &
    pids+=($!)
done
rc=0
for pid in "${pids[@]}"; do wait "$pid" || rc=$?; done
echo "exit $rc"
exit $rc
