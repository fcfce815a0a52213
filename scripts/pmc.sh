#!/bin/bash
# HBM traffic counters of the stream kernels, one counter group per rocprofv3
# pass (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass on gfx950).
# Usage: scripts/pmc.sh NAME [bench args...]
set -u
name=$1; shift
export TMPDIR=/tmp
for ctr in FETCH_SIZE WRITE_SIZE; do
  mkdir -p gpurun_out/$name/$ctr
  timeout -k 10 600 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/$name/$ctr -o run \
    -- python3 bench.py --no-cpu-baseline --no-latency "$@" > gpurun_out/$name/$ctr/bench.log 2>&1 || { echo "pmc $ctr failed rc=$?"; exit 1; }
done
echo "pmc ok" >&2
