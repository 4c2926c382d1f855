#!/bin/bash
# rank 0 of a 2-rank reduce_scatter_block probe under one rocprofv3 --pmc pass
export TMPDIR=/tmp
P=2; N=$1; CNT="$2"; OUT=$3
PORT=$((20000 + RANDOM % 20000))
mkdir -p "$OUT"
export MSX_SIZE=$P MSX_DEVICE=0 MSX_BOOTSTRAP_ADDR=127.0.0.1 MSX_BOOTSTRAP_PORT=$PORT MSX_BOOTSTRAP_TIMEOUT=90
MSX_RANK=0 timeout -s KILL 90 rocprofv3 --pmc $CNT -d "$OUT/prof" -o r0 --output-format csv -- python3 scripts/allreduce_probe.py "$N" 10 ${KIND:-rsb} > "$OUT/r0.log" 2>&1 &
a=$!
MSX_RANK=1 timeout -k 10 90 python3 scripts/allreduce_probe.py "$N" 10 ${KIND:-rsb} > "$OUT/r1.log" 2>&1 &
b=$!
wait $a; ra=$?; wait $b; rb=$?
exit $((ra | rb))
