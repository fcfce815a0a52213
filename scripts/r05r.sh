#!/bin/bash
# round-5 pass r: chain sub-phase stamps (config 4)
set -u
mkdir -p gpurun_out
KOORDHIP_STAMPS=1 timeout -k 10 300 python bench.py --workload config4 --steps 1 --warmup 1 --no-cpu-baseline > /dev/null 2> gpurun_out/r05r_stamps.err || { tail -5 gpurun_out/r05r_stamps.err; exit 1; }
grep "stamps\]" gpurun_out/r05r_stamps.err | grep -E "resolve cycles|chained|overlap|loop cycles" | tail -4 | cut -c1-400
