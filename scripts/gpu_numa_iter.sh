#!/bin/bash
# NodeNUMAResource iteration: every NUMA / topology / reservation GPU test, then config-3 stamps and bench
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "numa or topology or reservation or resv or config3 or launch_modes or rccl or kat" > gpurun_out/numa_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/numa_pytest.log; [ $rc -eq 0 ] || exit $rc
STAMP_WORKLOADS=config3 bash scripts/stamps.sh || exit 1
WORKLOAD=config3 BATCHES='12 16' bash scripts/sweep_batch.sh || exit 1
