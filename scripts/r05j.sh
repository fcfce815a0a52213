#!/bin/bash
# round-5 pass j: device-pod worker -- parity, config4dsmix with stamps
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_deviceshare.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r05j_ds.log 2>&1
rc=$?; tail -3 gpurun_out/r05j_ds.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|error|assert" gpurun_out/r05j_ds.log | head -30; tail -40 gpurun_out/r05j_ds.log; exit $rc; }
timeout -k 10 300 python bench.py --workload config4dsmix --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r05j_dsmix.json 2> gpurun_out/r05j_dsmix.err || { tail -20 gpurun_out/r05j_dsmix.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r05j_dsmix.json'));print('dsmix', d['value'], d['ms_per_step'])"
KOORDHIP_STAMPS=1 timeout -k 10 300 python bench.py --workload config4dsmix --steps 1 --warmup 1 --no-cpu-baseline > /dev/null 2> gpurun_out/r05j_dsmix_stamps.err || exit 1
grep "stamps\]" gpurun_out/r05j_dsmix_stamps.err | grep -E "device pods|resolve cycles" | tail -4 | cut -c1-400
timeout -k 10 300 python bench.py --workload deviceshare --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r05j_ds.json 2> gpurun_out/r05j_ds.err || { tail -20 gpurun_out/r05j_ds.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r05j_ds.json'));print('deviceshare', d['value'], d['ms_per_step'])"
