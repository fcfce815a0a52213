#!/bin/bash
# One rocprofv3 --pmc pass of SQ counters over a serial bench run (wave-time
# split of the stream kernels: active / issue-stalled / parked).
# Usage: CTRS="SQ_WAVES ..." scripts/sqpmc.sh NAME [bench args...]
set -u
name=$1; shift
export TMPDIR=/tmp
CTRS=${CTRS:-"SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU"}
mkdir -p gpurun_out/$name
KOORDHIP_SERIAL=1 timeout -s KILL 300 rocprofv3 --pmc $CTRS --output-format csv -d gpurun_out/$name -o run \
  -- python3 bench.py --no-cpu-baseline --no-latency "$@" > gpurun_out/$name/bench.log 2>&1 || { echo "sqpmc failed rc=$?"; exit 1; }
python3 - gpurun_out/$name <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for p in f:
    for r in csv.DictReader(open(p)):
        k = r["Kernel_Name"][:60]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        if r["Counter_Name"] == "SQ_WAVES": n[k] += 1
for k, d in sorted(acc.items(), key=lambda x: -x[1].get("SQ_WAVE_CYCLES", 0))[:6]:
    print(k, "launches", n[k], {c: round(v / max(n[k], 1)) for c, v in d.items()})
PY
