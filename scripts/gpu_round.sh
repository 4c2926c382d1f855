#!/bin/bash
# One GPU-box session: smoke, GPU parity tests, bench, rocprofv3 kernel trace.
# Stops at the first crash/timeout (exit codes other than 0 and 1).
cd "$(dirname "$0")/.." || exit 2
OUT=gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # step <name> <timeout_s> cmd...
    local name=$1 t=$2; shift 2
    echo "[$(date +%T)] start $name" | tee -a "$OUT/steps.log"
    timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "[$(date +%T)] end $name rc=$rc" | tee -a "$OUT/steps.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "abort after $name (rc=$rc)"; exit $rc; fi
    return 0
}
MODE=${1:-all}
rocm-smi --showproductname > "$OUT/rocm_smi.log" 2>&1
lscpu > "$OUT/lscpu.log" 2>&1; nproc >> "$OUT/lscpu.log"
if [ "$MODE" = all ] || [ "$MODE" = test ]; then
    step smoke 400 python -c "import __graft_entry__ as g; g.smoke()"
    step pytest_gpu 1200 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
    step bench 600 python bench.py --sweep
    # N = 2 with both ranks on this box's one GPU: exercises the N > 1 bench
    # path and the collectives harness (shared HBM, not xGMI)
    MSX_BENCH_LOG=$OUT/collectives_n2.log step bench_n2 600 python -m torch.distributed.run --nnodes=1 \
        --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29555 bench.py --gpus 2 --steps 20 --warmup 5
    step rocprof_trace 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_trace" -o trace --output-format csv -- python bench.py
    step rocprof_pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE -d "$OUT/prof_pmc" -o pmc_fetch --output-format csv -- python bench.py --steps 10 --warmup 2 --cpu-seconds 0.5 --no-host-path
    step rocprof_pmc_write 600 rocprofv3 --pmc WRITE_SIZE -d "$OUT/prof_pmc" -o pmc_write --output-format csv -- python bench.py --steps 10 --warmup 2 --cpu-seconds 0.5 --no-host-path
fi
echo done
