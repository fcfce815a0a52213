#!/bin/bash
# round-5 pass u: chains on / off for config 3 (NUMA build) and config 5
set -u
mkdir -p gpurun_out
for v in on off on off; do
  if [ $v = off ]; then export KOORDHIP_CHAIN_OFF=1; else unset KOORDHIP_CHAIN_OFF; fi
  timeout -k 10 300 python bench.py --workload config3 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r05u_c3_$v.json 2> gpurun_out/r05u.err || { tail -5 gpurun_out/r05u.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r05u_c3_$v.json'));print('config3 chain $v', d['value'], d['ms_per_step'])"
done
