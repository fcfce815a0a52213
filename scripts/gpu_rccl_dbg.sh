#!/bin/bash
set -u
mkdir -p gpurun_out
ldd koordinator_amd/lib/libkoordhip.so | grep -E "rccl|amdhip" > gpurun_out/rccl_ldd.txt
NCCL_DEBUG=INFO timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "rccl" > gpurun_out/rccl_dbg.log 2>&1
tail -3 gpurun_out/rccl_dbg.log
exit 0
