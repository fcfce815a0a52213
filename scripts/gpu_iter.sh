#!/bin/bash
# Iteration pass on the GPU box: GPU parity tests (optionally a -k filter),
# the config-4 bench with resolve stamps and without, then a rocprofv3
# kernel-stats pass (PROFILE=name).  Each GPU step is time-limited; the first
# failure stops the script.
set -u
mkdir -p gpurun_out
K=${TESTS_K:-}
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > gpurun_out/iter_tests.log 2>&1
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/iter_tests.log 2>&1
fi
rc=$?; tail -15 gpurun_out/iter_tests.log; [ $rc -eq 0 ] || exit $rc
KOORDHIP_STAMPS=1 timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/iter_stamps.json 2> gpurun_out/iter_stamps.err || exit $?
grep "stamps" gpurun_out/iter_stamps.err | tail -4
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/iter_bench.json 2> gpurun_out/iter_bench.err || exit $?
cut -c1-300 gpurun_out/iter_bench.json
if [ -n "${PROFILE:-}" ]; then
  bash scripts/profile.sh $PROFILE --steps 2 --warmup 1 ${BENCH_ARGS:-} || exit $?
  python3 - "$PROFILE" <<'PY'
import csv, glob, sys
f = glob.glob(f"gpurun_out/{sys.argv[1]}/**/*kernel_stats.csv", recursive=True)
for row in csv.DictReader(open(f[0])):
    print(row["Name"][:60], row["Calls"], row["AverageNs"], row["Percentage"])
PY
fi
