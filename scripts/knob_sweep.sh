#!/bin/bash
# A/B of library builds x environment knobs x round sizes on one workload
# (bench only; every run time-limited, the first failure stops the sweep).
# Usage: scripts/knob_sweep.sh WORKLOAD "KNOB=V ..." [bench args...]
#   LIBS="base wpe4"  library builds (base = koordinator_amd/lib/libkoordhip.so,
#                     else libkoordhip_<name>.so from `make variant`)
#   BATCHES="16 24"   round sizes (--batch), default the engine's
#   KNOB=V: "X=1" = the defaults
set -u
w=$1; knobs=$2; shift 2
out=gpurun_out/knobs_$w
mkdir -p $out
for lib in ${LIBS:-base}; do
  if [ "$lib" = base ]; then lp=koordinator_amd/lib/libkoordhip.so; else lp=koordinator_amd/lib/libkoordhip_$lib.so; fi
  for b in ${BATCHES:-0}; do
    for kv in $knobs; do
      tag=${lib}_b${b}_$kv
      env KOORDHIP_LIB=$lp $kv timeout -k 10 300 python bench.py --workload $w --steps ${STEPS:-2} --warmup 1 --no-cpu-baseline \
        --batch $b "$@" > $out/$tag.json 2> $out/$tag.err || { echo "failed $tag"; tail -3 $out/$tag.err; exit 1; }
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], 'P', d['config']['batch_pods'], 'eval', d['eval_roofline']['avg_launch_us'], 'select', d['select']['avg_launch_us'])" $out/$tag.json $tag
    done
  done
done
