#!/bin/bash
# round-5 pass l: config4dsmix repeated (the worker / class-list residency diagnostics on a stall)
set -u
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 120 python bench.py --workload config4dsmix --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r05l_$i.json 2> gpurun_out/r05l_$i.err || { grep -v "^ " gpurun_out/r05l_$i.err | tail -4; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r05l_$i.json'));print('run $i', d['value'], d['ms_per_step'])"
done
