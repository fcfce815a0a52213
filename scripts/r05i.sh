#!/bin/bash
# round-5 pass i: device pods inside the pipelined greedy (k_ext_worker) -- parity, then config4dsmix
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_deviceshare.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r05i_ds.log 2>&1
rc=$?; tail -5 gpurun_out/r05i_ds.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|error|assert" gpurun_out/r05i_ds.log | head -30; tail -40 gpurun_out/r05i_ds.log; exit $rc; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "place_stream_bit_exact or config2 or unschedulable or commit_uncommit or plugin_subsets or launch_modes" \
  --timeout 200 --timeout-method thread > gpurun_out/r05i_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r05i_pytest.log; [ $rc -eq 0 ] || { tail -60 gpurun_out/r05i_pytest.log; exit $rc; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -q -k "config4" --timeout 250 --timeout-method thread > gpurun_out/r05i_full.log 2>&1
rc=$?; tail -3 gpurun_out/r05i_full.log; [ $rc -eq 0 ] || { tail -60 gpurun_out/r05i_full.log; exit $rc; }
timeout -k 10 300 python bench.py --workload config4dsmix --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r05i_dsmix.json 2> gpurun_out/r05i_dsmix.err || { tail -20 gpurun_out/r05i_dsmix.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r05i_dsmix.json'));print('dsmix', d['value'], d['ms_per_step'], d.get('device_pods'))"
KOORDHIP_STAMPS=1 timeout -k 10 300 python bench.py --workload config4dsmix --steps 1 --warmup 1 --no-cpu-baseline > /dev/null 2> gpurun_out/r05i_dsmix_stamps.err || exit 1
grep "stamps\]" gpurun_out/r05i_dsmix_stamps.err | tail -12 | cut -c1-300
KOORDHIP_EXT_SEQ=1 timeout -k 10 300 python bench.py --workload config4dsmix --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r05i_dsmix_seq.json 2> gpurun_out/r05i_dsmix_seq.err || { tail -20 gpurun_out/r05i_dsmix_seq.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r05i_dsmix_seq.json'));print('dsmix sequential cycle', d['value'], d['ms_per_step'])"
timeout -k 10 300 python bench.py --workload config4 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r05i_c4.json 2> gpurun_out/r05i_c4.err || { tail -20 gpurun_out/r05i_c4.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r05i_c4.json'));print('config4', d['value'], d['ms_per_step'])"
timeout -k 10 300 python bench.py --workload deviceshare --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r05i_ds.json 2> gpurun_out/r05i_ds.err || { tail -20 gpurun_out/r05i_ds.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r05i_ds.json'));print('deviceshare', d['value'], d['ms_per_step'], d['config']['parallelism'])"
