#!/bin/bash
# P ranks sharing GPU 0 run scripts/allreduce_probe.py; rank 0 under rocprofv3
# kernel trace when PROF=1.  Usage: scripts/allreduce_probe.sh P NBYTES ITERS OUTDIR [KIND]
P=$1; N=$2; IT=$3; OUT=${4:-gpurun_out/arp}; KIND=${5:-allreduce}
PORT=$((20000 + RANDOM % 20000))
mkdir -p "$OUT"
pids=()
for ((r = 0; r < P; r++)); do
  export MSX_SIZE=$P MSX_RANK=$r MSX_DEVICE=0 MSX_BOOTSTRAP_ADDR=127.0.0.1 MSX_BOOTSTRAP_PORT=$PORT MSX_BOOTSTRAP_TIMEOUT=90
  if [ "$r" = 0 ] && [ "${PROF:-0}" = 1 ]; then
    timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o r0 -- python3 scripts/allreduce_probe.py "$N" "$IT" "$KIND" > "$OUT/r$r.log" 2>&1 &
  else
    timeout -k 10 180 python3 scripts/allreduce_probe.py "$N" "$IT" "$KIND" > "$OUT/r$r.log" 2>&1 &
  fi
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait "$p" || rc=$?; done
cat "$OUT"/r*.log | grep rank
exit $rc
