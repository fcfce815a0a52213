#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 120 --timeout-method thread -k "not config3 and not config2" > gpurun_out/r2d_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r2d_pytest.log; [ $rc -eq 0 ] || exit $rc
BATCHES='24' bash scripts/sweep_batch.sh || exit 1
STAMP_WORKLOADS=config4 bash scripts/stamps.sh
