#!/bin/bash
# round-5 pass p: the Reservation builds without the chain masks -- config 5 parity + bench
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -q -k "config5" --timeout 500 --timeout-method thread > gpurun_out/r05p_full.log 2>&1
rc=$?; tail -2 gpurun_out/r05p_full.log; [ $rc -eq 0 ] || { tail -40 gpurun_out/r05p_full.log; exit $rc; }
timeout -k 10 300 python bench.py --workload config5 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r05p_c5.json 2> gpurun_out/r05p_c5.err || { tail -20 gpurun_out/r05p_c5.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r05p_c5.json'));print('config5', d['value'], d['ms_per_step'], 'P', d['config']['batch_pods'])"
