export TMPDIR=/tmp
for n in 4096 1048576 16777216; do
  bash scripts/allreduce_probe.sh 4 $n 30 gpurun_out/sc_$n scan > gpurun_out/sc_${n}_fl.txt 2>&1 || exit 1
  MSX_RD_FLAGS=0 bash scripts/allreduce_probe.sh 4 $n 30 gpurun_out/scn_$n scan > gpurun_out/sc_${n}_hb.txt 2>&1 || exit 1
done
