#!/bin/bash
# k_eval_topk slice width (KOORDHIP_ETK_VT) x pipeline lag on config 5.
set -u
mkdir -p gpurun_out
for lag in X=1 KOORDHIP_LAG2=1; do
  for vt in 8 16 32; do
    env $lag KOORDHIP_ETK_VT=$vt timeout -k 10 300 python bench.py --workload ${W:-config5} --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/vt_${vt}_$lag.json 2> gpurun_out/vt_${vt}_$lag.err || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['eval_roofline']['avg_launch_us'], d['config']['batch_pods'], d['config']['pipeline_lag'])" gpurun_out/vt_${vt}_$lag.json "VT=$vt $lag"
  done
done
