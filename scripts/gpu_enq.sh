#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 200 python scripts/enqueue_time.py > gpurun_out/enq.log 2>&1 || exit 1
timeout -k 10 200 python scripts/enqueue_time.py comm >> gpurun_out/enq.log 2>&1 || exit 1
grep enqueue gpurun_out/enq.log
