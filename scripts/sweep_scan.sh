#!/bin/bash
# k_scan shape sweep (bench only): KOORDHIP_TOPK_R nodes per lane x KOORDHIP_SCAN_PW pods per wave.
set -u
mkdir -p gpurun_out
for cfg in ${SWEEP:-"1 2" "1 4" "2 1" "2 2" "2 4" "4 1" "4 2"}; do
  set -- $cfg
  KOORDHIP_TOPK_R=$1 KOORDHIP_SCAN_PW=$2 timeout -k 10 120 python bench.py --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/sweep_$1_$2.json 2>/dev/null || exit $?
  python3 -c "import json,sys; d=json.load(open('gpurun_out/sweep_$1_$2.json')); print('R=$1 pw=$2', d['value'], d['eval_roofline']['avg_launch_us'], d['select']['avg_launch_us'])"
done
