#!/bin/bash
# round-5 pass o: chain passes A/B (config 4) + parity of the default
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "place_stream_bit_exact or config2 or unschedulable or commit_uncommit or plugin_subsets or launch_modes" \
  --timeout 200 --timeout-method thread > gpurun_out/r05o_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r05o_pytest.log; [ $rc -eq 0 ] || { tail -60 gpurun_out/r05o_pytest.log; exit $rc; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -q -k "config4" --timeout 250 --timeout-method thread > gpurun_out/r05o_full.log 2>&1
rc=$?; tail -2 gpurun_out/r05o_full.log; [ $rc -eq 0 ] || { tail -60 gpurun_out/r05o_full.log; exit $rc; }
for v in 3 2 1 3; do
  KOORDHIP_CHAIN_PASSES=$v timeout -k 10 300 python bench.py --workload config4 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r05o_c4_$v.json 2> gpurun_out/r05o_c4.err || { tail -20 gpurun_out/r05o_c4.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r05o_c4_$v.json'));print('passes $v', d['value'], d['ms_per_step'])"
done
KOORDHIP_STAMPS=1 timeout -k 10 300 python bench.py --workload config4 --steps 1 --warmup 1 --no-cpu-baseline > /dev/null 2> gpurun_out/r05o_stamps.err || exit 1
grep "stamps\]" gpurun_out/r05o_stamps.err | grep -E "resolve cycles|chained|overlap" | tail -3 | cut -c1-300
