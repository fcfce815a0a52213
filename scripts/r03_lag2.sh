#!/bin/bash
# Lag 2 for the NUMA / Reservation plugin sets (KOORDHIP_LAG2): parity of the
# side-configuration streams, then bench lines of configs 5 / 3 at lag 1 and 2.
set -u
mkdir -p gpurun_out
KOORDHIP_LAG2=1 timeout -k 10 900 python -u -m pytest ${LAG2_TESTS:-tests/test_gpu_reservation.py tests/test_gpu_numa.py tests/test_reservation_slots.py tests/test_resv_cpus.py tests/test_gpu_topology_policy.py} -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/lag2_tests.log 2>&1
rc=$?; tail -3 gpurun_out/lag2_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/lag2_tests.log | head; exit $rc; }
for w in config5 config3; do
  for v in X=1 KOORDHIP_LAG2=1; do
    env $v timeout -k 10 300 python bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/lag2_${w}_$v.json 2> gpurun_out/lag2_${w}_$v.err || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['eval_roofline']['avg_launch_us'], d.get('round_pods'), d.get('lag'))" gpurun_out/lag2_${w}_$v.json "$w $v"
  done
done
