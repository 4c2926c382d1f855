#!/bin/bash
# P ranks sharing GPU 0, EVERY rank under rocprofv3 --kernel-trace (timeline
# comparison).  Usage: scripts/prof_both.sh P NBYTES ITERS OUTDIR KIND
export TMPDIR=/tmp
P=$1; N=$2; IT=$3; OUT=$4; KIND=${5:-allreduce}
PORT=$((20000 + RANDOM % 20000))
mkdir -p "$OUT"
pids=()
for ((r = 0; r < P; r++)); do
  MSX_SIZE=$P MSX_RANK=$r MSX_DEVICE=0 MSX_BOOTSTRAP_ADDR=127.0.0.1 MSX_BOOTSTRAP_PORT=$PORT MSX_BOOTSTRAP_TIMEOUT=90 \
    timeout -k 10 180 rocprofv3 --kernel-trace -d "$OUT/prof" -o r$r -- python3 scripts/allreduce_probe.py "$N" "$IT" "$KIND" > "$OUT/r$r.log" 2>&1 &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait "$p" || rc=$?; done
exit $rc
