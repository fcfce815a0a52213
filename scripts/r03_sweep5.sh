#!/bin/bash
# config 5 (200k nodes, reservations holding CPUs, NUMA) round size sweep at lag 2 on the final round-3 build
set -u
mkdir -p gpurun_out
run() {
  tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --workload config5 --steps 2 --warmup 1 --no-cpu-baseline $ARGS > gpurun_out/sw5_$tag.json 2> gpurun_out/sw5_$tag.err || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['eval_roofline']['avg_launch_us'])" gpurun_out/sw5_$tag.json "$tag"
}
for b in 32 20 24 28; do
  ARGS="--batch $b" run b${b} X=1
done
ARGS="--batch 32" run b32_again X=1
