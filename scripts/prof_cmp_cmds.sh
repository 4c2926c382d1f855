export TMPDIR=/tmp
PROF=1 bash scripts/allreduce_probe.sh 2 2097152 20 gpurun_out/pc_rs2 rsb > gpurun_out/pc_rs2.txt 2>&1 || exit 1
MSX_RS_VIA_OUT=1 PROF=1 bash scripts/allreduce_probe.sh 2 2097152 20 gpurun_out/pc_rs2o rsb > gpurun_out/pc_rs2o.txt 2>&1 || exit 1
MSX_RS_VIA_OUT=1 bash scripts/allreduce_probe.sh 4 1048576 20 gpurun_out/pc_rs4o rsb > gpurun_out/pc_rs4o.txt 2>&1 || exit 1
