#!/bin/bash
# Iteration pass: a GPU test selection (TESTS_FILES / TESTS_K; SKIP_TESTS=1 for
# none), then bench lines (no CPU baseline) of WORKLOADS under each
# environment variant in VARIANTS ("X=1" = the defaults).  Time-limited steps;
# the first failure stops the script.
set -u
mkdir -p gpurun_out
FILES=${TESTS_FILES:-"tests/test_gpu_parity.py tests/test_gpu_reservation.py tests/test_gpu_numa.py tests/test_fit_kat.py"}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest $FILES -m gpu -x -q --timeout 120 --timeout-method thread ${TESTS_K:+-k "$TESTS_K"} > gpurun_out/iter_tests.log 2>&1
  rc=$?; tail -25 gpurun_out/iter_tests.log; [ $rc -eq 0 ] || exit $rc
fi
for w in ${WORKLOADS:-config4 config5 config3}; do
  for v in ${VARIANTS:-X=1}; do
    tag=$(echo "$v" | tr '/' '_')
    env $v timeout -k 10 300 python bench.py --workload $w --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} \
      > gpurun_out/iter_${w}_${tag}.json 2> gpurun_out/iter_${w}_${tag}.err
    rc=$?
    python3 - gpurun_out/iter_${w}_${tag}.json "$w $v" <<'PY'
import json, sys
try:
    d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
    print(sys.argv[2], "pods/s", d["value"], "ms/step", d["ms_per_step"], "eval", d["eval_roofline"].get("avg_launch_us", d["eval_roofline"].get("avg_launch_ms")),
          "select us", d.get("select", {}).get("avg_launch_us"), "unsched", d["unschedulable"])
except Exception as e:
    print(sys.argv[2], "no result", e)
PY
    [ $rc -eq 0 ] || { tail -20 gpurun_out/iter_${w}_${tag}.err; exit $rc; }
    if [ "${STAMPS:-0}" = 1 ]; then
      env $v KOORDHIP_STAMPS=1 timeout -k 10 300 python bench.py --workload $w --steps 1 --warmup 1 --no-cpu-baseline --no-latency ${BENCH_ARGS:-} \
        > /dev/null 2> gpurun_out/iter_stamps_${w}_${tag}.err || exit 1
      grep "stamps\] \(resolve cycles\|round\|device\)" gpurun_out/iter_stamps_${w}_${tag}.err | tail -4 | cut -c1-400
    fi
  done
done
exit 0
