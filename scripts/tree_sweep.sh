# tree kernel sweep at deployment sizes: per-source size x
# mode; every probe is one short process with its own limit
set -e
mkdir -p gpurun_out/tree/sweep4
for mib in 32 48 64 128; do
  TREE_MIB=$mib TREE_MODES=0,4,12 TREE_CAPS=0 timeout -k 10 120 python scripts/tree_probe.py > gpurun_out/tree/sweep4/m${mib}.json 2>> gpurun_out/tree/sweep4/err.log
  echo "done $mib"
done
