#!/bin/bash
# round-5 pass k: the device-pod worker's CU partition A/B (config4dsmix)
set -u
mkdir -p gpurun_out
for v in default nocstream nomask; do
  case $v in nocstream) export KOORDHIP_EXT_NOCSTREAM=1;; nomask) export KOORDHIP_EXT_NOMASK=1;; esac
  timeout -k 10 120 python bench.py --workload config4dsmix --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r05k_$v.json 2> gpurun_out/r05k_$v.err || { tail -5 gpurun_out/r05k_$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r05k_$v.json'));print('$v', d['value'], d['ms_per_step'], d['eval_roofline'].get('avg_launch_ms'))"
  unset KOORDHIP_EXT_NOCSTREAM KOORDHIP_EXT_NOMASK
done
