#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2f_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r2f_pytest.log; [ $rc -eq 0 ] || exit $rc
BATCHES='24' bash scripts/sweep_batch.sh || exit 1
WORKLOAD=config5 BATCHES='16 32' bash scripts/sweep_batch.sh || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/sweep_config5_16.json')); print(d['eval_roofline']['avg_launch_us'], d['select'])"
