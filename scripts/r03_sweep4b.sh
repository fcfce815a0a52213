#!/bin/bash
# config 4 knob combinations (after r03_sweep4.sh): select workgroups x scan nodes per lane
set -u
mkdir -p gpurun_out
run() {
  tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/sw4b_$tag.json 2> gpurun_out/sw4b_$tag.err || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['eval_roofline']['avg_launch_us'], d['select']['avg_launch_us'])" gpurun_out/sw4b_$tag.json "$tag"
}
run default X=1
run g6 KOORDHIP_SEL_G=6
run r4 KOORDHIP_TOPK_R=4
run g6r4 KOORDHIP_SEL_G=6 KOORDHIP_TOPK_R=4
run g5r4 KOORDHIP_SEL_G=5 KOORDHIP_TOPK_R=4
run g4r4 KOORDHIP_SEL_G=4 KOORDHIP_TOPK_R=4
run g7r4 KOORDHIP_SEL_G=7 KOORDHIP_TOPK_R=4
run default2 X=1
run g6r4b KOORDHIP_SEL_G=6 KOORDHIP_TOPK_R=4
