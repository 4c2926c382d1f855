# k_combine_dram: correctness (every pair, forced) and the size sweep of the
# default dispatch before/after
set -e
mkdir -p gpurun_out/mall/dram
timeout -k 10 400 python -u -m pytest -x -q --timeout 380 --timeout-method thread tests/test_gpu_local.py -k "dram or maximum_count or beyond_4gib or benchmark_size" > gpurun_out/mall/dram/tests.log 2>&1
MALL_SIZES=256,512,1024,2048 timeout -k 10 200 python scripts/mall_probe.py > gpurun_out/mall/dram/probe.json 2>/dev/null
MSX_COMBINE_DRAM_MIN=1099511627776 MALL_SIZES=512,1024,2048 timeout -k 10 200 python scripts/mall_probe.py > gpurun_out/mall/dram/probe_old.json 2>/dev/null
