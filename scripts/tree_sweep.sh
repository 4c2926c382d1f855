# tree kernel: default dispatch vs plain / non-temporal loads around the
# 256 MiB source-bytes bound
set -e
mkdir -p gpurun_out/tree/sweep6
for mib in 32 48 64; do
  TREE_MIB=$mib TREE_MODES=0,4,12 TREE_CAPS=0 timeout -k 10 120 python scripts/tree_probe.py > gpurun_out/tree/sweep6/m${mib}.json 2>> gpurun_out/tree/sweep6/err.log
done
