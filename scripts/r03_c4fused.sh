#!/bin/bash
# config 4: the split scan + select vs the fused k_eval_topk at VT = 4 / 8 (and G = 2 at VT = 4)
set -u
mkdir -p gpurun_out
for v in X=1 "KOORDHIP_EVAL=fused KOORDHIP_ETK_VT=4" "KOORDHIP_EVAL=fused KOORDHIP_ETK_VT=8" "KOORDHIP_EVAL=fused KOORDHIP_ETK_VT=4 KOORDHIP_ETK_G=2"; do
  tag=$(echo "$v" | tr ' =' '_-')
  env $v timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/c4f_$tag.json 2> gpurun_out/c4f_$tag.err || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['eval_roofline']['kernel'], d['eval_roofline']['avg_launch_us'], d['select']['avg_launch_us'])" gpurun_out/c4f_$tag.json "$v"
done
