#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "rccl or launch_modes" > gpurun_out/r2b_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r2b_pytest.log; [ $rc -eq 0 ] || exit $rc
bash scripts/stamps.sh
