#!/bin/bash
# Run GPU steps in order, each under its own time limit, logging to
# gpurun_out/<name>.log.  A step that ends by a signal, an abort or a time
# limit (exit >= 124) stops the sequence: nothing more touches the GPU after a
# fault or a hang.  Plain failures (pytest rc 1) let the next step run.
# Usage: scripts/gpu_steps.sh "name|seconds|command" ...
mkdir -p gpurun_out
worst=0
for spec in "$@"; do
    name=${spec%%|*}; rest=${spec#*|}; secs=${rest%%|*}; cmd=${rest#*|}
    echo "== $name (limit ${secs}s): $cmd"
    timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
    rc=$?
    tail -n 6 "gpurun_out/$name.log"
    echo "== $name rc=$rc"
    [ $rc -gt $worst ] && worst=$rc
    if [ $rc -ge 124 ]; then
        echo "== stopping: $name ended with $rc"
        exit $rc
    fi
done
exit $worst
