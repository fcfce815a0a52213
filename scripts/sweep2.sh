#!/bin/bash
# Tuning sweep of the config-4 stream over split-select groups (KOORDHIP_SEL_G),
# round size (--batch) and scan unroll (KOORDHIP_TOPK_R); bench only, no profiler.
# Every run has its own time limit; the first failure stops the sweep.
set -u
mkdir -p gpurun_out/sweep2
for G in ${GS:-4 8 16}; do
  for B in ${BS:-24 32 48}; do
    for R in ${RS:-2 4}; do
      log=gpurun_out/sweep2/${WL:-config4}_g${G}_b${B}_r${R}.log
      KOORDHIP_SEL_G=$G KOORDHIP_TOPK_R=$R timeout -k 10 120 python bench.py --no-cpu-baseline --workload ${WL:-config4} --steps 2 --warmup 1 \
        --batch $B > $log 2>&1 || { echo "G=$G B=$B R=$R failed rc=$?"; tail -3 $log; exit 1; }
      python - "$G" "$B" "$R" $log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[4]) if l.startswith('{')][-1])
print(f"G={sys.argv[1]} B={sys.argv[2]} R={sys.argv[3]} pods/s={d['value']:.0f} ms/step={d['ms_per_step']:.1f} "
      f"scan_us={d['roofline']['avg_launch_us']}", flush=True)
PY
    done
  done
done
