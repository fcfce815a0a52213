#!/bin/bash
# round-5 pass b: the class-incremental lists -- parity first, then config 4
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "place_stream_bit_exact or config2 or unschedulable or commit_uncommit or plugin_subsets or launch_modes" \
  --timeout 200 --timeout-method thread > gpurun_out/r05b_pytest.log 2>&1
rc=$?; tail -5 gpurun_out/r05b_pytest.log; [ $rc -eq 0 ] || { tail -80 gpurun_out/r05b_pytest.log; exit $rc; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -q -k "config4" --timeout 250 --timeout-method thread > gpurun_out/r05b_full.log 2>&1
rc=$?; tail -5 gpurun_out/r05b_full.log; [ $rc -eq 0 ] || { tail -60 gpurun_out/r05b_full.log; exit $rc; }
timeout -k 10 300 python bench.py --workload config4 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r05b_c4.json 2> gpurun_out/r05b_c4.err || { tail -20 gpurun_out/r05b_c4.err; exit 1; }
tail -c 900 gpurun_out/r05b_c4.json
KOORDHIP_STAMPS=1 timeout -k 10 300 python bench.py --workload config4 --steps 1 --warmup 1 --no-cpu-baseline > /dev/null 2> gpurun_out/r05b_c4_stamps.err || exit 1
grep "stamps\]" gpurun_out/r05b_c4_stamps.err | tail -8 | cut -c1-250
