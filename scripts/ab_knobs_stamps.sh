#!/bin/bash
# Env-knob A/B on one workload: bench value + resolve stamps per knob setting.
# Usage: W=config4 KNOBS="X=1 KOORDHIP_CU_RESERVE=1" bash scripts/ab_knobs_stamps.sh
set -u
mkdir -p gpurun_out
w=${W:-config4}
for v in ${KNOBS:-X=1}; do
  env $v timeout -k 10 300 python bench.py --workload $w --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline > gpurun_out/k_$v.json 2>/dev/null || { echo "failed $v"; exit 1; }
  echo "== $v $(grep -o '"value": [0-9.]*' gpurun_out/k_$v.json | head -1)"
  if [ "${NOSTAMPS:-0}" != 1 ]; then
    env $v KOORDHIP_STAMPS=1 timeout -k 10 300 python bench.py --workload $w --steps 1 --warmup 1 --no-cpu-baseline > /dev/null 2> gpurun_out/k_$v.err || exit 1
    grep "stamps\] \(resolve\|prologue\)" gpurun_out/k_$v.err | cut -c1-260
  fi
done
