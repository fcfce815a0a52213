#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2c_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r2c_pytest.log; [ $rc -eq 0 ] || exit $rc
for w in config4 config5; do
  timeout -k 10 300 python bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline --one-rank-comm > gpurun_out/r2c_comm1_$w.json 2> gpurun_out/r2c_comm1_$w.err || { echo "bench $w failed"; tail -5 gpurun_out/r2c_comm1_$w.err; exit 1; }
  cut -c1-400 gpurun_out/r2c_comm1_$w.json
done
