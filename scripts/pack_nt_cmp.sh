#!/bin/bash
# A/B of the datatype pack/unpack kernels with plain (default) vs non-temporal
# typed-side accesses (MSX_DT_TYPED_NT=1, a variant since removed: see DESIGN 3b): bench.py pack table.
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out/pack_nt
for i in 0 1; do
  for NT in 0 1; do
    MSX_DT_TYPED_NT=$NT timeout -k 10 120 python bench.py --steps 5 --warmup 2 --cpu-seconds 0.2 --no-host-path \
      --no-per-op --no-collectives > gpurun_out/pack_nt/r${i}_nt${NT}.json 2> gpurun_out/pack_nt/r${i}_nt${NT}.err || exit 1
  done
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/pack_nt/*.json")):
    d = json.load(open(f))["datatype_pack_roofline_hbm"]
    print(f.split("/")[-1], {k: (v["pack"]["us"], v["unpack"]["us"]) for k, v in d.items()})
PY
