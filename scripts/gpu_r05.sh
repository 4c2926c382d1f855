#!/bin/bash
# Round-5 GPU session: smoke, the whole GPU suite (default environment), the
# N = 1 bench, then (MODE=all) the N = 2 shared-GPU bench.  Every step under its
# own time limit; stops at the first step that crashes or times out.
# Usage: scripts/gpu_r05.sh OUTDIR [test|bench|all]
cd "$(dirname "$0")/.." || exit 2
OUT=${1:-gpurun_out/r05}
MODE=${2:-all}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # step <name> <timeout_s> cmd...
    local name=$1 t=$2; shift 2
    echo "[$(date +%T)] start $name" | tee -a "$OUT/steps.log"
    timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "[$(date +%T)] end $name rc=$rc" | tee -a "$OUT/steps.log"
    tail -n 2 "$OUT/$name.log"
    [ $rc -eq 0 ] || { echo "abort after $name (rc=$rc)"; exit $rc; }
}
if [ "$MODE" = all ] || [ "$MODE" = test ]; then
    step smoke 400 python -c "import __graft_entry__ as g; g.smoke()"
    step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
    step bench_n1 600 python bench.py
fi
if [ "$MODE" = all ]; then
    MSX_BENCH_LOG=$OUT/collectives_n2.log step bench_n2 600 python -m torch.distributed.run --nnodes=1 \
        --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29555 bench.py --gpus 2 --steps 20 --warmup 5
fi
