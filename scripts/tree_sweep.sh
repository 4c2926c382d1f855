# tree kernel: non-temporal loads x tile order at deployment sizes
set -e
mkdir -p gpurun_out/tree/sweep5
for mib in 64 128; do
  TREE_MIB=$mib TREE_MODES=0,14 TREE_CAPS=0 TREE_ORDERS=0,2147483647,32,128 timeout -k 10 120 python scripts/tree_probe.py > gpurun_out/tree/sweep5/m${mib}.json 2>> gpurun_out/tree/sweep5/err.log
  echo "done $mib"
done
