#!/bin/bash
# Round-size sweep on the GPU box: bench lines per batch_pods (config 4 and 3).
set -u
mkdir -p gpurun_out
W=${WORKLOAD:-config4}
for b in ${BATCHES:-24 32 48 64}; do
  timeout -k 10 240 python bench.py --workload $W --steps 3 --warmup 1 --no-cpu-baseline --batch $b \
    > gpurun_out/sweep_${W}_$b.json 2> gpurun_out/sweep_${W}_$b.err || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'])" \
    gpurun_out/sweep_${W}_$b.json $b
done
