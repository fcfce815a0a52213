#!/bin/bash
set -u
mkdir -p gpurun_out
KOORDHIP_STAMPS=1 timeout -k 10 300 python bench.py --workload config4 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r05d.json 2> gpurun_out/r05d_stamps.err || { tail gpurun_out/r05d_stamps.err; exit 1; }
grep "stamps\]" gpurun_out/r05d_stamps.err | tail -9 | cut -c1-300
