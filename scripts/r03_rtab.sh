#!/bin/bash
# Key tables for the reservation-matched pods: parity of the reservation files +
# the full-size config-5 fixture, then config 5 with and without them (same box).
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_reservation.py tests/test_reservation_slots.py tests/test_resv_cpus.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 600 --timeout-method thread -k "resv or slot or config5 or reserv" > gpurun_out/rtab_tests.log 2>&1
rc=$?; tail -3 gpurun_out/rtab_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/rtab_tests.log | head; exit $rc; }
for v in X=1 KOORDHIP_NO_RESV_TABLES=1 X=2 KOORDHIP_NO_RESV_TABLES=2; do
  env $v timeout -k 10 300 python bench.py --workload config5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/rtab_$v.json 2> gpurun_out/rtab_$v.err || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/rtab_$v.json "$v"
done
KOORDHIP_STAMPS=1 timeout -k 10 300 python bench.py --workload config5 --steps 1 --warmup 1 --no-cpu-baseline > /dev/null 2> gpurun_out/rtab_stamps.err || exit 1
grep "stamps" gpurun_out/rtab_stamps.err | head -8
