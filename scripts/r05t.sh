#!/bin/bash
# round-5 pass t: device-pod hand-off split (config4dsmix stamps)
set -u
mkdir -p gpurun_out
KOORDHIP_STAMPS=1 timeout -k 10 300 python bench.py --workload config4dsmix --steps 1 --warmup 1 --no-cpu-baseline > /dev/null 2> gpurun_out/r05t_stamps.err || { tail -5 gpurun_out/r05t_stamps.err; exit 1; }
grep "device pods" gpurun_out/r05t_stamps.err | tail -1 | cut -c1-700
