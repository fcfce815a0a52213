#!/bin/bash
# config 4 knob re-sweep on the final round-3 build: select workgroups per pod,
# scan nodes per lane, round size (bench --batch)
set -u
mkdir -p gpurun_out
run() {
  tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline $EXTRA > gpurun_out/sw4_$tag.json 2> gpurun_out/sw4_$tag.err || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['eval_roofline']['avg_launch_us'], d['select']['avg_launch_us'], d['config']['batch_pods'])" gpurun_out/sw4_$tag.json "$tag"
}
EXTRA=""
run default X=1
for g in 6 8 12 16; do run selg$g KOORDHIP_SEL_G=$g; done
for r in 1 4; do run topkr$r KOORDHIP_TOPK_R=$r; done
for b in 20 28; do EXTRA="--batch $b"; run batch$b X=1; done
EXTRA=""
run default2 X=1
