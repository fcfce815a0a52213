#!/bin/bash
# config-4 sweep of round size x lag on the class-list pipeline
set -u
mkdir -p gpurun_out
for v in X=1 KOORDHIP_LAG1=1; do
  for b in ${BATCHES:-16 20 24 28 32}; do
    env $v timeout -k 10 200 python bench.py --workload config4 --steps 3 --warmup 1 --no-cpu-baseline --batch $b \
      > gpurun_out/r05f_${v}_$b.json 2> gpurun_out/r05f_${v}_$b.err || { tail -5 gpurun_out/r05f_${v}_$b.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'], d['config']['batch_pods'], d['config']['pipeline_lag'])" gpurun_out/r05f_${v}_$b.json $v $b
  done
done
