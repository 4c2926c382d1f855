#!/bin/bash
# Round 5, DESIGN.md §2: try once to catch a pageable-transfer hole in the act.
# The whole GPU suite first (the host / device memory churn both round-4
# reproductions had behind them), then the 8-rank stress cases with the
# harness's transfers pageable (MSX_TEST_PINNED=0, sentinels on) for two
# passes of the 240-call loop, under round 4's reproduction knobs.  A hole
# then shows as `where_wrong`'s "N hold the readback sentinel" / "own send
# buffer N wrong" with the device result correct.  Read once, not repeated.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
out=gpurun_out/r05_catch
mkdir -p "$out"
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 400 \
    --timeout-method thread > "$out/suite.log" 2>&1
rc=$?; echo "suite rc=$rc"; tail -n 2 "$out/suite.log"; [ $rc -eq 0 ] || exit $rc
export MSX_TEST_PINNED=0 MSX_STRESS_PASSES=2 MSX_CHUNK_BYTES=536870912 MSX_PUSH_VECS=1024 \
       MSX_PUSH_GRID_CAP=2048 MSX_COMBINE_DRAM_MIN=268435457 MSX_COPY_DRAM_MIN=268435457
timeout -k 10 560 python -u -m pytest -q -p no:cacheprovider --timeout 540 --timeout-method thread \
    "tests/test_gpu_multirank.py::test_collectives_p_ranks_on_one_gpu[8-None-None-+ts]" \
    "tests/test_gpu_multirank.py::test_collectives_p_ranks_on_one_gpu[8-None-None-switch0+ts]" \
    > "$out/stress.log" 2>&1
rc=$?; echo "stress rc=$rc"; tail -n 2 "$out/stress.log"
exit 0
