#!/bin/bash
# A/B of library builds x environment knobs on one workload (bench only; each
# run time-limited, the first failure stops the sweep).
# Usage: scripts/ab_libs.sh WORKLOAD "LIBNAME ..." "KNOB=V ..." [bench args...]
#   LIBNAME: "base" = koordinator_amd/lib/libkoordhip.so, else libkoordhip_<LIBNAME>.so
#   KNOB=V:  "X=1" = the defaults
set -u
w=$1; libs=$2; knobs=$3; shift 3
out=gpurun_out/ab_$w
mkdir -p $out
for lib in $libs; do
  if [ "$lib" = base ]; then lp=koordinator_amd/lib/libkoordhip.so; else lp=koordinator_amd/lib/libkoordhip_$lib.so; fi
  for kv in $knobs; do
    tag=${lib}_$kv
    env KOORDHIP_LIB=$lp $kv timeout -k 10 300 python bench.py --workload $w --steps ${STEPS:-2} --warmup 1 --no-cpu-baseline "$@" \
      > $out/$tag.json 2> $out/$tag.err || { echo "failed $tag"; tail -3 $out/$tag.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], 'P', d['config']['batch_pods'], 'scan', d['eval_roofline']['avg_launch_us'], 'select', d['select']['avg_launch_us'])" $out/$tag.json $tag
  done
done
