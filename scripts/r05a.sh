#!/bin/bash
# round-5 pass a: the new ABI-12 tests, the k_seq exit under rocprofv3, a config-4 baseline
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_deviceshare.py tests/test_reserve_pods.py -m gpu -x -q \
  --timeout 200 --timeout-method thread > gpurun_out/r05a_pytest.log 2>&1
rc=$?; tail -5 gpurun_out/r05a_pytest.log; [ $rc -eq 0 ] || { tail -60 gpurun_out/r05a_pytest.log; exit $rc; }
bash scripts/profile.sh r05a_spread --workload spread --steps 1 --warmup 1
rc=$?; tail -3 gpurun_out/r05a_spread/bench.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload config4 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r05a_c4.json 2> gpurun_out/r05a_c4.err || exit 1
tail -c 600 gpurun_out/r05a_c4.json
KOORDHIP_STAMPS=1 timeout -k 10 300 python bench.py --workload config4 --steps 1 --warmup 1 --no-cpu-baseline > /dev/null 2> gpurun_out/r05a_c4_stamps.err || exit 1
grep "stamps\]" gpurun_out/r05a_c4_stamps.err | tail -8 | cut -c1-250
