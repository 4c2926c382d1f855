#!/bin/bash
# all GPU tests, N=1 bench (host paths), N=2 shared-GPU bench with uncached and cached windows
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py > gpurun_out/n1.json 2> gpurun_out/n1.err || { echo "bench n1 rc=$?"; tail -20 gpurun_out/n1.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/n1.json')); print(d['value'], d['roofline']['frac'], json.dumps(d.get('host_path')))"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29600 bench.py --gpus 2 --steps 5 --warmup 2 --no-host-path > gpurun_out/n2u.json 2> gpurun_out/n2u.err || { echo "bench u rc=$?"; tail -20 gpurun_out/n2u.err; exit 1; }
MSX_WINDOW_CACHED=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29601 bench.py --gpus 2 --steps 5 --warmup 2 --no-host-path > gpurun_out/n2c.json 2> gpurun_out/n2c.err || { echo "bench c rc=$?"; tail -20 gpurun_out/n2c.err; exit 1; }
python - <<'PY'
import json
for f in ("gpurun_out/n2u.json", "gpurun_out/n2c.json"):
    d = json.load(open(f))
    print(f, json.dumps(d["collectives"]))
PY
