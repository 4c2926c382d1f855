mkdir -p gpurun_out/lat
for i in 0 1; do
timeout -k 10 60 python scripts/latency_probe.py 3000 >> gpurun_out/lat/lat.jsonl || exit 1
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 60 python scripts/latency_probe.py 3000 >> gpurun_out/lat/lat.jsonl || exit 1
MSX_PROBE_SPIN=1 timeout -k 10 60 python scripts/latency_probe.py 3000 >> gpurun_out/lat/lat.jsonl || exit 1
MSX_PROBE_SPIN=1 HIP_FORCE_DEV_KERNARG=1 timeout -k 10 60 python scripts/latency_probe.py 3000 >> gpurun_out/lat/lat.jsonl || exit 1
done
cat gpurun_out/lat/lat.jsonl
