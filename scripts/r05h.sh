#!/bin/bash
# round-5 pass h: chained staged decisions in the resolve -- parity, then A/B with KOORDHIP_CHAIN on and off
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "place_stream_bit_exact or config2 or unschedulable or commit_uncommit or plugin_subsets or launch_modes" \
  --timeout 200 --timeout-method thread > gpurun_out/r05h_pytest.log 2>&1
rc=$?; tail -5 gpurun_out/r05h_pytest.log; [ $rc -eq 0 ] || { tail -80 gpurun_out/r05h_pytest.log; exit $rc; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -q -k "config4" --timeout 250 --timeout-method thread > gpurun_out/r05h_full.log 2>&1
rc=$?; tail -5 gpurun_out/r05h_full.log; [ $rc -eq 0 ] || { tail -60 gpurun_out/r05h_full.log; exit $rc; }
for v in on off on off; do
  if [ $v = off ]; then export KOORDHIP_CHAIN_OFF=1; else unset KOORDHIP_CHAIN_OFF; fi
  timeout -k 10 300 python bench.py --workload config4 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r05h_c4_$v.json 2> gpurun_out/r05h_c4.err || { tail -20 gpurun_out/r05h_c4.err; exit 1; }
  echo "chain $v: $(python -c "import json;d=json.load(open('gpurun_out/r05h_c4_$v.json'));print(d['value'],d['ms_per_step'])")"
done
unset KOORDHIP_CHAIN_OFF
KOORDHIP_STAMPS=1 timeout -k 10 300 python bench.py --workload config4 --steps 1 --warmup 1 --no-cpu-baseline > /dev/null 2> gpurun_out/r05h_stamps.err || exit 1
grep "stamps\]" gpurun_out/r05h_stamps.err | tail -9 | cut -c1-300
