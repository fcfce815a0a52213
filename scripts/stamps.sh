#!/bin/bash
# resolve / select cycle stamps (KOORDHIP_STAMPS) of configs 4 and 3, one step each
set -u
mkdir -p gpurun_out
for w in ${STAMP_WORKLOADS:-config4 config3}; do
  KOORDHIP_STAMPS=1 timeout -k 10 300 python bench.py --workload $w --steps 1 --warmup 1 --no-cpu-baseline \
    > gpurun_out/stamps_$w.json 2> gpurun_out/stamps_$w.err || { echo "failed $w"; exit 1; }
  grep stamps gpurun_out/stamps_$w.err | tail -6
done
