#!/bin/bash
# c3-c5 harness (bench_collectives.py) with 2 ranks sharing GPU 0 at full size,
# three engine settings in one job: the round-3 schedule (host-barrier chunks
# above 256 MiB: MSX_TWO_STEP_MAX=268435456), the round-4 GPU-flag pipeline
# (default, one stream), the pipeline with the collect overlapped
# (MSX_COLLECT_OVERLAP=1), and the first two with a 960 MiB window chunk.
# Usage: scripts/c3_pipeline_ab.sh OUTDIR
OUT=${1:-gpurun_out/c3ab}
mkdir -p "$OUT"
cd "$(dirname "$0")/.." || exit 2
for round in 1 2; do
  for cfg in ${CONFIGS:-"r03|MSX_TWO_STEP_MAX=268435456" "pipe|MSX_NOTHING=0" "overlap|MSX_COLLECT_OVERLAP=1" "r03_c960|MSX_TWO_STEP_MAX=268435456 MSX_CHUNK_BYTES=1006632960" "pipe_c960|MSX_CHUNK_BYTES=1006632960"}; do
    name=${cfg%%|*}; kv=${cfg#*|}
    PORT=$((20000 + RANDOM % 20000))
    pids=()
    for r in 0 1; do
      env $kv MSX_SIZE=2 MSX_RANK=$r MSX_DEVICE=0 MSX_BOOTSTRAP_ADDR=127.0.0.1 MSX_BOOTSTRAP_PORT=$PORT \
          MSX_BOOTSTRAP_TIMEOUT=120 timeout -k 10 200 python bench_collectives.py "$OUT/${name}_r$round.json" 1.0 \
          > "$OUT/${name}_r${round}_rank$r.out" 2>&1 &
      pids+=($!)
    done
    rc=0
    for pid in "${pids[@]}"; do wait "$pid" || rc=$?; done
    [ $rc -ne 0 ] && { echo "$name round $round rc=$rc"; tail -5 "$OUT/${name}_r${round}_rank0.out"; exit $rc; }
    python3 - "$OUT/${name}_r$round.json" "$name" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
def g(k):
    v = d.get(k) or {}
    return f"{k.split('_')[0]} {v.get('seconds', v.get('ms'))} s correct={v.get('correct')}"
print(sys.argv[2], "|", " | ".join(g(k) for k in ("c3_allreduce_sum_f32", "c4_reduce_scatter_max_f64", "c5_iallreduce_band_u64")), flush=True)
PY
  done
done
