#!/bin/bash
set -u
mkdir -p gpurun_out
bash scripts/profile.sh r05c_c4 --workload config4 --steps 1 --warmup 1 || exit 1
head -12 gpurun_out/r05c_c4/run_kernel_stats.csv | cut -c1-200
python3 - <<'PY'
import csv, collections
rows = list(csv.DictReader(open("gpurun_out/r05c_c4/run_kernel_trace.csv")))
by = collections.defaultdict(list)
for r in rows:
    by[r["Kernel_Name"][:40]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for k, v in by.items():
    v.sort()
    print(k, len(v), "p50", v[len(v)//2], "p90", v[int(len(v)*0.9)], "max", v[-1])
PY
