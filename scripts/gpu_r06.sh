#!/bin/bash
# Round-6 GPU session steps, each under its own time limit; stops at the first
# step that fails, crashes or times out.  Libraries are built beforehand, in
# this tree, on the CPU container.
# Usage: scripts/gpu_r06.sh OUTDIR MODE
#   MODE test      smoke + the whole GPU suite
#   MODE bench     the N = 1 bench
#   MODE rehearse  N = 8 ranks on this box's one GPU, the variant run enabled
#                  (MSX_BENCH_VARIANTS_AT=8) and rank 3's IPC core child hung
#                  on the host (MSX_BENCH_TEST_HANG), under a 300 s wall budget
#   MODE prof      rocprofv3 kernel trace + stats of a short N = 1 bench
cd "$(dirname "$0")/.." || exit 2
OUT=${1:-gpurun_out/r06}
MODE=${2:-test}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # step <name> <timeout_s> cmd...
    local name=$1 t=$2; shift 2
    echo "[$(date +%T)] start $name" | tee -a "$OUT/steps.log"
    timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "[$(date +%T)] end $name rc=$rc" | tee -a "$OUT/steps.log"
    tail -n 3 "$OUT/$name.log"
    [ $rc -eq 0 ] || { echo "abort after $name (rc=$rc)"; exit $rc; }
}
case "$MODE" in
test)
    step smoke 400 python -c "import __graft_entry__ as g; g.smoke()"
    step pytest_gpu 1000 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread \
        -p no:cacheprovider
    ;;
bench)
    step bench_n1 600 python bench.py
    ;;
rehearse)
    MSX_BENCH_VARIANTS_AT=8 MSX_BENCH_TEST_HANG=ipc:3 MSX_BENCH_WALL_S=300 MSX_BENCH_LOG=$OUT/coll_n8.log \
        step bench_n8_hang 420 python bench.py --gpus 8 --steps 20 --warmup 5
    ;;
prof)
    step prof_n1 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o n1 --output-format csv -- \
        python bench.py --steps 50 --warmup 10 --no-host-path --no-per-op --no-pack --no-collectives --cpu-seconds 1
    ;;
*) echo "unknown mode $MODE"; exit 2 ;;
esac
