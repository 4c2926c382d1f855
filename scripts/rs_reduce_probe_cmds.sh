export TMPDIR=/tmp
for kind in rsb reduce; do
  for n in 1048576 16777216 67108864; do
    bash scripts/allreduce_probe.sh 4 $n 30 gpurun_out/p_${kind}_$n $kind > gpurun_out/p_${kind}_${n}_fl.txt 2>&1 || exit 1
    MSX_TWO_STEP_MAX=0 bash scripts/allreduce_probe.sh 4 $n 30 gpurun_out/pn_${kind}_$n $kind > gpurun_out/p_${kind}_${n}_hb.txt 2>&1 || exit 1
  done
done
