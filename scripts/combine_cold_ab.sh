# interleaved A/B of the combine candidates, cache cold and warm
set -e
mkdir -p gpurun_out/mall/ab
SWEEP_ROUNDS=5 SWEEP_COLD=1 SWEEP_SIZES=256 SWEEP_VARIANTS=0,7,23,20,24 timeout -k 10 200 python scripts/combine_size_sweep.py > gpurun_out/mall/ab/cold256.json 2>/dev/null
SWEEP_ROUNDS=5 SWEEP_SIZES=256,1024 SWEEP_VARIANTS=0,7,23,20,24 timeout -k 10 200 python scripts/combine_size_sweep.py > gpurun_out/mall/ab/warm.json 2>/dev/null
