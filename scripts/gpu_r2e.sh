#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2e_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r2e_pytest.log; [ $rc -eq 0 ] || exit $rc
BATCHES='24' bash scripts/sweep_batch.sh || exit 1
WORKLOAD=config3 BATCHES='16' bash scripts/sweep_batch.sh || exit 1
STAMP_WORKLOADS=config4 bash scripts/stamps.sh
