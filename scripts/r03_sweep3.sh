#!/bin/bash
# config 3 (NUMA cpusets) round size x pipeline lag sweep on the final round-3 build
set -u
mkdir -p gpurun_out
run() {
  tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --workload config3 --steps 3 --warmup 1 --no-cpu-baseline $ARGS > gpurun_out/sw3_$tag.json 2> gpurun_out/sw3_$tag.err || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['eval_roofline']['avg_launch_us'])" gpurun_out/sw3_$tag.json "$tag"
}
for b in 16 8 12 20 24 32; do
  ARGS="--batch $b" run b${b}_lag1 X=1
  ARGS="--batch $b" run b${b}_lag2 KOORDHIP_LAG2=1
done
ARGS="--batch 16" run b16_lag1_again X=1
