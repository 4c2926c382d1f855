#!/bin/bash
# multirank + RMA GPU tests, then N=2 (shared GPU) bench with uncached and cached engine windows
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_multirank.py tests/test_gpu_rma.py -x -q > gpurun_out/mr.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/mr.log; exit 1; }
tail -2 gpurun_out/mr.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29600 bench.py --gpus 2 --steps 5 --warmup 2 --no-host-path > gpurun_out/n2u.json 2> gpurun_out/n2u.err || { echo "bench u rc=$?"; tail -20 gpurun_out/n2u.err; exit 1; }
MSX_WINDOW_CACHED=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29601 bench.py --gpus 2 --steps 5 --warmup 2 --no-host-path > gpurun_out/n2c.json 2> gpurun_out/n2c.err || { echo "bench c rc=$?"; tail -20 gpurun_out/n2c.err; exit 1; }
python - <<'PY'
import json
for f in ("gpurun_out/n2u.json", "gpurun_out/n2c.json"):
    d = json.load(open(f))
    print(f, json.dumps(d["collectives"]))
PY
