#!/bin/bash
# Datatype GPU tests, then bench.py's pack table with the two-level compact
# form off (MSX_DT_COMPACT2=0: explicit run tables) and on (default), alternating.
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out/compact2
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_dtype.py tests/test_gpu_dtype_multirank.py tests/test_gpu_rma.py tests/test_gpu_rma_passive.py \
    > gpurun_out/compact2/tests.log 2>&1 || { tail -30 gpurun_out/compact2/tests.log; exit 1; }
tail -2 gpurun_out/compact2/tests.log
for i in 0 1; do
  for C2 in 0 1; do
    MSX_DT_COMPACT2=$C2 timeout -k 10 120 python bench.py --steps 5 --warmup 2 --cpu-seconds 0.2 --no-host-path \
      --no-per-op --no-collectives > gpurun_out/compact2/r${i}_c${C2}.json 2> gpurun_out/compact2/r${i}_c${C2}.err || exit 1
  done
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/compact2/*.json")):
    d = json.load(open(f))["datatype_pack_roofline_hbm"]
    print(f.split("/")[-1], {k: (v["pack"]["us"], v["unpack"]["us"], v["pack"]["kernel"]) for k, v in d.items()})
PY
