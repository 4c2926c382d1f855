#!/bin/bash
# Generic tree kernel in the DRAM regime: A/B of mode 3 (non-temporal, 256-lane
# grid-stride, the earlier default), 17 (one-wave dispatch order, the new
# default) and 0 (default dispatch: the compile-time kernel for p = 8), per-source
# 64 and 128 MiB; then the tree / multirank parity suites with non-temporal
# trees forced on.  usage: scripts/tree_generic_check.sh OUTDIR
cd "$(dirname "$0")/.." || exit 2
OUT=${1:-gpurun_out/tree_generic}
mkdir -p "$OUT"
set -o pipefail
for mib in 64 128; do
  TREE_MIB=$mib TREE_MODES=0,3,8,17 TREE_CAPS=0 timeout -k 10 180 python scripts/tree_probe.py > "$OUT/tree_${mib}.json" 2> "$OUT/tree_${mib}.err" || exit 3
done
echo "tree probes done"
timeout -k 10 300 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_gpu_local.py -k tree > "$OUT/local_tree.log" 2>&1 || { tail -20 "$OUT/local_tree.log"; exit 4; }
tail -1 "$OUT/local_tree.log"
MSX_TREE_NT_MIN=0 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_local.py tests/test_gpu_multirank.py tests/test_gpu_nbc.py -k "tree or multirank or nbc or allreduce or reduce" > "$OUT/forced_nt.log" 2>&1 || { tail -20 "$OUT/forced_nt.log"; exit 5; }
tail -1 "$OUT/forced_nt.log"
