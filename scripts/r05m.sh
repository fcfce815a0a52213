#!/bin/bash
# round-5 pass m: config4dsmix repeated -- the worker on a pooled stream (default) vs a dedicated queue
set -u
mkdir -p gpurun_out
for i in 1 2 3 4 5; do
  timeout -k 10 120 python bench.py --workload config4dsmix --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r05m_$i.json 2> gpurun_out/r05m_$i.err || { grep -v "^ " gpurun_out/r05m_$i.err | cut -c1-300 | tail -3; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r05m_$i.json'));print('pooled run $i', d['value'], d['ms_per_step'])"
done
