# round-3 kernels forced on everywhere: non-temporal tree loads for every
# tree launch (MSX_TREE_NT_MIN=0) and the DRAM-regime combine for every
# device combine (MSX_COMBINE_DRAM_MIN=0), through the local and multi-rank
# parity suites
set -e
mkdir -p gpurun_out/stress_r03
export MSX_TREE_NT_MIN=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_gpu_local.py -k tree > gpurun_out/stress_r03/tree_nt_local.log 2>&1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_multirank.py tests/test_gpu_nbc.py > gpurun_out/stress_r03/tree_nt_multirank.log 2>&1
unset MSX_TREE_NT_MIN
MSX_COMBINE_DRAM_MIN=0 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_local.py tests/test_gpu_op_table.py > gpurun_out/stress_r03/combine_dram.log 2>&1
