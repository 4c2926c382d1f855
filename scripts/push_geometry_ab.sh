#!/bin/bash
# Why the pipelined reduce_scatter rounds (c4) run slower than the host-barrier
# rounds with 2 ranks on one GPU: the push geometry and store policy.  The c3/c4
# harness with: host-barrier rounds, the pipeline as is, the pipeline with plain
# stores (MSX_WT_STORES=0), the pipeline with the copy kernel's one-tile-per-
# workgroup grid (MSX_PUSH_VECS=256 MSX_PUSH_GRID_CAP=65536), both.
cd "$(dirname "$0")/.." || exit 2
OUT=${1:-gpurun_out/pushab}
mkdir -p "$OUT"
for round in 1 2; do
  for cfg in "hb|MSX_TWO_STEP_MAX=268435456" "pipe|MSX_NOTHING=0" "pipe_plain|MSX_WT_STORES=0" \
             "pipe_grid|MSX_PUSH_VECS=256 MSX_PUSH_GRID_CAP=65536" \
             "pipe_grid_plain|MSX_PUSH_VECS=256 MSX_PUSH_GRID_CAP=65536 MSX_WT_STORES=0"; do
    name=${cfg%%|*}; kv=${cfg#*|}
    PORT=$((20000 + RANDOM % 20000))
    pids=()
    for r in 0 1; do
      env $kv MSX_COLL_ONLY=c3c4 MSX_SIZE=2 MSX_RANK=$r MSX_DEVICE=0 MSX_BOOTSTRAP_ADDR=127.0.0.1 \
          MSX_BOOTSTRAP_PORT=$PORT MSX_BOOTSTRAP_TIMEOUT=120 timeout -k 10 200 \
          python bench_collectives.py "$OUT/${name}_r$round.json" 1.0 > "$OUT/${name}_r${round}_rank$r.out" 2>&1 &
      pids+=($!)
    done
    rc=0
    for pid in "${pids[@]}"; do wait "$pid" || rc=$?; done
    [ $rc -ne 0 ] && { echo "$name round $round rc=$rc"; tail -5 "$OUT/${name}_r${round}_rank0.out"; exit $rc; }
    python3 - "$OUT/${name}_r$round.json" "$name" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
c3, c4 = d.get("c3_allreduce_sum_f32") or {}, d.get("c4_reduce_scatter_max_f64") or {}
print(sys.argv[2], "| c3", c3.get("seconds"), c3.get("correct"), "| c4", c4.get("seconds"), c4.get("correct"), flush=True)
PY
  done
done
