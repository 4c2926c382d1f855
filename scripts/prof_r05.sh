#!/bin/bash
# Round-5 profiles of the headline kernel: rocprofv3 kernel
# trace + stats, then FETCH_SIZE and WRITE_SIZE in separate --pmc passes (the
# guide's HBM section: FETCH_SIZE x 2 on gfx950), each over the N = 1 bench.
# MODE=all also runs one whole GPU suite under round 4's reproduction
# conditions with the page-locked test harness.
# Usage: scripts/prof_r05.sh OUTDIR [prof|r3|all]
cd "$(dirname "$0")/.." || exit 2
OUT=${1:-gpurun_out/r05prof}
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
B="bench.py --no-host-path --no-per-op --no-pack --no-collectives --cpu-seconds 1"
if [ "$MODE" = all ] || [ "$MODE" = prof ]; then
    step prof_trace 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o trace --output-format csv -- python $B
    step pmc_fetch 180 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o pmc_fetch --output-format csv -- python $B
    step pmc_write 180 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o pmc_write --output-format csv -- python $B
fi
if [ "$MODE" = all ] || [ "$MODE" = r3 ]; then
    MSX_TWO_STEP_MAX=4611686018427387904 MSX_CHUNK_BYTES=536870912 MSX_PUSH_VECS=1024 MSX_PUSH_GRID_CAP=2048 \
    MSX_COMBINE_DRAM_MIN=268435457 MSX_COPY_DRAM_MIN=268435457 \
        step suite_r3_conditions 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread \
        -p no:cacheprovider
fi
