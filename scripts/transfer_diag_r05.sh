#!/bin/bash
# Round 5, DESIGN.md §2: ONE job of two whole GPU suites under the conditions
# of round 4's two reproductions (flag schedules forced on, round-3 window
# layout, 512 MiB chunk, round-3 push geometry and combine / copy thresholds),
# with the harness's transfers pageable (MSX_TEST_PINNED=0) as they were then.
# Each pageable transfer lands on a sentinel and every stress mismatch is
# located (device result, readback, the rank's own upload) by the worker's
# where_wrong().  Evidence collection, read once; not a rate estimate.
# (Ran with the round-4 library build and the round-5 worker; MSX_WINDOW_LAYOUT was removed
# from the library after this run and is ignored since.)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
out=gpurun_out/r05_diag
mkdir -p "$out"
export MSX_TEST_PINNED=0 MSX_TWO_STEP_MAX=4611686018427387904 MSX_WINDOW_LAYOUT=1 \
       MSX_CHUNK_BYTES=536870912 MSX_PUSH_VECS=1024 MSX_PUSH_GRID_CAP=2048 \
       MSX_COMBINE_DRAM_MIN=268435457 MSX_COPY_DRAM_MIN=268435457
for s in A B; do
    timeout -k 10 540 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider \
        --timeout 400 --timeout-method thread > "$out/suite$s.log" 2>&1
    rc=$?
    echo "suite $s rc=$rc"
    tail -n 3 "$out/suite$s.log"
    [ $rc -eq 0 ] || exit $rc
done
