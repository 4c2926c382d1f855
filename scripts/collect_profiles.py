"""Copy the judged evidence of a scripts/gpu_round.sh run from gpurun_out/
(scratch) into profiles/<round>/ (tracked): bench JSON lines, the rocprofv3
kernel statistics, the kernel trace rows of the timed kernels, PMC counters."""
import csv
import json
import os
import shutil
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "gpurun_out")
DST = os.path.join(REPO, "profiles", sys.argv[1] if len(sys.argv) > 1 else "r01")
os.makedirs(DST, exist_ok=True)


def json_line(log):
    with open(os.path.join(SRC, log)) as f:
        lines = [x for x in f if x.startswith('{"metric"')]
    return json.loads(lines[-1]) if lines else None


for log, name in (("bench.log", "bench_n1.json"), ("rocprof_trace.log", "bench_n1_under_rocprof.json"),
                  ("bench_n2.log", "bench_n2_shared_gpu.json")):
    if not os.path.exists(os.path.join(SRC, log)):
        continue
    d = json_line(log)
    if d:
        with open(os.path.join(DST, name), "w") as f:
            json.dump(d, f, indent=1)
with open(os.path.join(SRC, "bench.log")) as f:
    sweep = [x for x in f if "GB/s" in x and not x.startswith("{")]
with open(os.path.join(DST, "bench_sweep.log"), "w") as f:
    f.writelines(sweep)
shutil.copy(os.path.join(SRC, "prof_trace", "trace_kernel_stats.csv"), DST)
keep = ("k_combine_dram<3, float, float, 64, true, false>", "k_combine<3, float, float, 1, 256, true, false>", "k_dt_", "k_tree<3, float, float, 256, false, false, 8, 1, false>")
with open(os.path.join(SRC, "prof_trace", "trace_kernel_trace.csv")) as fi, \
        open(os.path.join(DST, "trace_kernel_trace.csv"), "w", newline="") as fo:
    r, w = csv.reader(fi), csv.writer(fo)
    hdr = next(r)
    w.writerow(hdr)
    k = hdr.index("Kernel_Name")
    for row in r:
        if any(s in row[k] for s in keep) and "k_combine_host" not in row[k]:
            w.writerow(row)
for n in ("pmc_fetch_counter_collection.csv", "pmc_write_counter_collection.csv"):
    with open(os.path.join(SRC, "prof_pmc", n)) as fi, open(os.path.join(DST, n), "w", newline="") as fo:
        r, w = csv.reader(fi), csv.writer(fo)
        hdr = next(r)
        w.writerow(hdr)
        k = hdr.index("Kernel_Name")
        for row in r:
            if any(s in row[k] for s in keep) and "k_combine_host" not in row[k]:
                w.writerow(row)
shutil.copy(os.path.join(SRC, "steps.log"), DST)
if os.path.exists(os.path.join(SRC, "collectives_n2.log")):
    shutil.copy(os.path.join(SRC, "collectives_n2.log"), os.path.join(DST, "collectives_n2_shared_gpu.log"))
print("profiles ->", DST)
