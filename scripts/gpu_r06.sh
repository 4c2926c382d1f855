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
#   MODE geom      the combine's launch geometries, warm and cold (scripts/combine_geometry_probe.py)
#   MODE measure   bench, geom, prof, then rehearse, in one session
#   MODE geom2     the geometry sweep at 8 MiB - 2 GiB, 5 rounds
#   MODE full      test, bench, geom2, treegeom, prof
#   MODE rehearse_clean  N = 8 on the one GPU, default sequence, nothing hung
#   MODE treegeom  the 8-source DRAM-regime tree in other tile orders (scripts/tree_geometry_probe.py)
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
run_mode() {
case "$1" in
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
    # kernel trace + stats of the default N = 1 bench command, then FETCH_SIZE
    # and WRITE_SIZE in separate --pmc passes (the guide's HBM section:
    # FETCH_SIZE x 2 on gfx950) over the device-side tables
    B="bench.py --no-host-path --no-collectives --cpu-seconds 1"
    step prof_trace 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o trace --output-format csv -- python bench.py
    step pmc_fetch 240 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o pmc_fetch --output-format csv -- python $B
    step pmc_write 240 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o pmc_write --output-format csv -- python $B
    ;;
geom)
    step geom 300 python scripts/combine_geometry_probe.py 64,256,1024 3
    ;;
geom2)
    step geom2 400 python scripts/combine_geometry_probe.py 8,16,32,64,128,256,512,1024,2048 5
    ;;
treegeom)
    step treegeom 300 python scripts/tree_geometry_probe.py 32,64,128 3
    ;;
rehearse_clean)
    # the default N = 8 sequence with every rank on this box's one GPU (no hang)
    MSX_BENCH_VARIANTS_AT=8 MSX_BENCH_LOG=$OUT/coll_n8_clean.log \
        step bench_n8_clean 500 python bench.py --gpus 8 --steps 20 --warmup 5
    ;;
measure)
    run_mode bench && run_mode geom && run_mode prof && run_mode rehearse
    ;;
full)
    run_mode test && run_mode bench && run_mode geom2 && run_mode treegeom && run_mode prof
    ;;
*) echo "unknown mode $1"; exit 2 ;;
esac
}
run_mode "$MODE"
