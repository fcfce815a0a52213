#!/bin/bash
# round-5 pass q: device-pod pre-evaluation lead A/B (config4dsmix) + DeviceShare parity
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_deviceshare.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r05q_ds.log 2>&1
rc=$?; tail -2 gpurun_out/r05q_ds.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/r05q_ds.log | head -20; exit $rc; }
for v in 2 5 8 5; do
  KOORDHIP_EXT_LEAD=$v timeout -k 10 300 python bench.py --workload config4dsmix --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r05q_$v.json 2> gpurun_out/r05q_$v.err || { tail -5 gpurun_out/r05q_$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r05q_$v.json'));print('lead $v', d['value'], d['ms_per_step'])"
done
KOORDHIP_STAMPS=1 timeout -k 10 300 python bench.py --workload config4dsmix --steps 1 --warmup 1 --no-cpu-baseline > /dev/null 2> gpurun_out/r05q_stamps.err || exit 1
grep "device pods" gpurun_out/r05q_stamps.err | tail -1 | cut -c1-400
timeout -k 10 300 python bench.py --workload deviceshare --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r05q_dsw.json 2> gpurun_out/r05q_dsw.err || { tail -5 gpurun_out/r05q_dsw.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r05q_dsw.json'));print('deviceshare', d['value'], d['ms_per_step'])"
