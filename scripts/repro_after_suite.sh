#!/bin/bash
# The round-3 wrong result appeared only in whole-suite runs,
# after the full-size and local suites had churned GBs of HBM.  Run those
# first, then ROUNDS fresh 8-rank replays of the multirank worker (one pass
# of the stress loop each, as in the suite), stopping at the first failure.
# Usage: scripts/repro_after_suite.sh ROUNDS [PASSES]
set -o pipefail
cd "$(dirname "$0")/.."
ROUNDS=${1:-6}
PASSES=${2:-1}
mkdir -p gpurun_out/repro
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_local.py -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/repro/preamble.log 2>&1
rc=$?
tail -3 gpurun_out/repro/preamble.log
[ $rc -eq 0 ] || { echo "preamble rc=$rc"; exit $rc; }
for i in $(seq 1 "$ROUNDS"); do
    timeout -k 10 300 python -u scripts/repro_stress.py 8 "$PASSES" > gpurun_out/repro/round$i.log 2>&1
    rc=$?
    tail -1 gpurun_out/repro/round$i.log
    if [ $rc -ne 0 ]; then
        cat gpurun_out/repro/round$i.log
        exit $rc
    fi
done
echo "no failure in $ROUNDS rounds"
