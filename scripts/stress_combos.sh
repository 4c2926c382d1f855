#!/bin/bash
# Moved MS-MPI switch points combined with the engine's protocol variants
# (multirank cases inherit the environment).  Output: gpurun_out/combos.log
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
: > gpurun_out/combos.log
run() {  # run <switch value> <pytest -k expr>
    echo "== switch=$1 case=$2" >> gpurun_out/combos.log
    MPICH_DEFAULT_ALLREDUCE_SHORT_MSG=$1 MPICH_DEFAULT_REDUCE_SHORT_MSG=$1 MPICH_DEFAULT_REDSCAT_COMMUTATIVE_LONG_MSG=$1 \
    timeout -k 10 300 python -u -m pytest -q --timeout 240 --timeout-method thread -p no:cacheprovider \
        tests/test_gpu_multirank.py -k "$2" >> gpurun_out/combos.log 2>&1
}
run 2147483647 "3-None-None-0" && run 0 "3-None-None-unfused" && run 0 "4-None-None-ts512k" && \
run 2147483647 "2-None-None-None" && run 0 "7-1048576-None-None" && run 2147483647 "4-65536-None-0"
rc=$?
grep -E "^==|passed|failed" gpurun_out/combos.log
exit $rc
