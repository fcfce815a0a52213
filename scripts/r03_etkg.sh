#!/bin/bash
# k_eval_topk pods-per-workgroup A/B: parity of the fused streams at G = 4,
# then bench lines of configs 5 / 3 at G = 1 / 2 / 4 and config 4 fused.
set -u
mkdir -p gpurun_out
KOORDHIP_ETK_G=4 timeout -k 10 600 python -u -m pytest tests/test_gpu_reservation.py tests/test_gpu_numa.py tests/test_reservation_slots.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/etkg_tests.log 2>&1
rc=$?; tail -3 gpurun_out/etkg_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/etkg_tests.log | head; exit $rc; }
for w in config5 config3; do
  for g in 1 2 4; do
    KOORDHIP_ETK_G=$g timeout -k 10 300 python bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/etkg_${w}_$g.json 2> gpurun_out/etkg_${w}_$g.err || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['eval_roofline']['avg_launch_us'])" gpurun_out/etkg_${w}_$g.json "$w G=$g"
  done
done
for g in 1 4; do
  KOORDHIP_EVAL=fused KOORDHIP_ETK_G=$g timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/etkg_config4_$g.json 2> gpurun_out/etkg_config4_$g.err || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['eval_roofline']['avg_launch_us'])" gpurun_out/etkg_config4_$g.json "config4 fused G=$g"
done
