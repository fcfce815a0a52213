#!/bin/bash
# configs 3 / 5 (and 4ds): the class lists vs the scan path
set -u
mkdir -p gpurun_out
for w in config3 config5 config4ds; do
  for v in X=1 KOORDHIP_CLS_OFF=1; do
    env $v timeout -k 10 300 python bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline \
      > gpurun_out/r05g_${w}_$v.json 2> gpurun_out/r05g_${w}_$v.err || { tail -5 gpurun_out/r05g_${w}_$v.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); e=d['eval_roofline']; print(sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'], e['kernel'], e.get('classes'), d['config']['batch_pods'], d['config']['pipeline_lag'])" gpurun_out/r05g_${w}_$v.json $w $v
  done
done
