#!/bin/bash
# One-sided, datatype and full-size paths with unusual knob values.
# Output: gpurun_out/knobs2.log
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
: > gpurun_out/knobs2.log
run() {  # run "<env assignments>" <test file> <-k expr>
    echo "== $1 :: $2 $3" >> gpurun_out/knobs2.log
    env $1 timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider \
        "$2" -k "$3" >> gpurun_out/knobs2.log 2>&1
}
run "MSX_RMA_BYTES=1048576" tests/test_gpu_rma_passive.py "" && \
run "MSX_RMA_BYTES=1048576" tests/test_gpu_rma_pscw.py "" && \
run "MSX_CHUNK_BYTES=8192" tests/test_gpu_rma.py "" && \
run "MSX_CHUNK_BYTES=8192" tests/test_gpu_rma_compact.py "" && \
run "MSX_CHUNK_BYTES=16384" tests/test_gpu_dtype_multirank.py "" && \
run "MSX_CHUNK_BYTES=67108864" tests/test_gpu_fullsize.py "c3-3 or c4-2"
rc=$?
grep -E "^==|passed|failed" gpurun_out/knobs2.log
exit $rc
