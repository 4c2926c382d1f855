#!/bin/bash
# The bench's RCCL reference point in its child process: 1 rank (RCCL runs),
# then 2 ranks sharing one GPU (RCCL refuses: must come back as an error entry).
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29710 timeout -k 10 150 python scripts/rccl_native_check.py || exit 1
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29720 scripts/rccl_native_check.py || exit 1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29730 bench.py --gpus 2 --steps 20 --warmup 5 > gpurun_out/n2_after_clock.json 2> gpurun_out/n2_after_clock.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/n2_after_clock.json')); print(d['value'], d['ms_per_step'], d['roofline']['kernel_us_mean_max_rank'])"
