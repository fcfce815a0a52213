#!/bin/bash
# A/B of environment knobs on one workload (bench only; every run time-limited,
# the first failure stops the sweep).
# Usage: scripts/knob_sweep.sh WORKLOAD "KNOB=V KNOB2=V2 ..." [bench args...]
#   e.g. scripts/knob_sweep.sh config5 "X=1 KOORDHIP_SEL_G=16 KOORDHIP_TOPK_R=1"
#   (X=1 = the defaults)
set -u
w=$1; knobs=$2; shift 2
out=gpurun_out/knobs_$w
mkdir -p $out
for kv in $knobs; do
  env $kv timeout -k 10 300 python bench.py --workload $w --steps ${STEPS:-2} --warmup 1 --no-cpu-baseline "$@" \
    > $out/$kv.json 2> $out/$kv.err || { echo "failed $kv"; tail -3 $out/$kv.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], 'P', d['config']['batch_pods'], 'scan', d['eval_roofline']['avg_launch_us'], 'select', d['select']['avg_launch_us'])" $out/$kv.json $kv
done
