#!/bin/bash
# Tuning sweep of the stream path (bench only, no profiler).
set -u
mkdir -p gpurun_out/sweep
for R in ${RS:-2 4 8}; do
  for B in ${BS:-32 64}; do
    KOORDHIP_TOPK_R=$R timeout -k 10 300 python bench.py --no-cpu-baseline --pods ${PODS:-20000} --steps 2 --warmup 1 --batch $B \
      > gpurun_out/sweep/r${R}_b${B}.log 2>&1 || { echo "R=$R B=$B failed rc=$?"; tail -3 gpurun_out/sweep/r${R}_b${B}.log; exit 1; }
    python - "$R" "$B" gpurun_out/sweep/r${R}_b${B}.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[3]) if l.startswith('{')][-1])
r = d['roofline']
print(f"R={sys.argv[1]} B={sys.argv[2]} pods/s={d['value']:.0f} ms/step={d['ms_per_step']:.1f} eval_us={r['avg_launch_us']} GB/s={r['achieved']}")
PY
  done
done
