#!/bin/bash
# Engine knobs at unusual but legal values, each over a multirank case that
# inherits the environment.  Output: gpurun_out/knobs.log
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
: > gpurun_out/knobs.log
run() {  # run "<env assignments>" <test file> <-k expr>
    echo "== $1 :: $3" >> gpurun_out/knobs.log
    env $1 timeout -k 10 300 python -u -m pytest -q --timeout 240 --timeout-method thread -p no:cacheprovider \
        "$2" -k "$3" >> gpurun_out/knobs.log 2>&1
}
run "MSX_CHUNK_BYTES=4096" tests/test_gpu_multirank.py "5-None-None-None" && \
run "MSX_CHUNK_BYTES=12288" tests/test_gpu_multirank.py "2-None-None-None" && \
run "MSX_TWO_STEP_MAX=0" tests/test_gpu_multirank.py "6-None-None-None" && \
run "MSX_HOST_BOUNCE_MAX=67108864" tests/test_gpu_multirank.py "5-None-None-None" && \
run "MSX_HOST_PIN_MIN=0" tests/test_gpu_multirank.py "5-None-None-None" && \
run "MPICH_DEFAULT_ALLREDUCE_SHORT_MSG=0 MPICH_DEFAULT_REDUCE_SHORT_MSG=0 MPICH_DEFAULT_REDSCAT_COMMUTATIVE_LONG_MSG=0" tests/test_gpu_comm_split.py "" && \
run "MSX_FUSED_PUSH=0 MPICH_DEFAULT_ALLREDUCE_SHORT_MSG=2147483647" tests/test_gpu_multirank.py "6-None-None-None"
rc=$?
grep -E "^==|passed|failed" gpurun_out/knobs.log
exit $rc
