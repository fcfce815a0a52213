#!/bin/bash
# round evidence: full GPU suite, then profiles + bench lines (scripts/profile_round.sh), config-5 bench
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/round_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/round_pytest.log; [ $rc -eq 0 ] || exit $rc
ROUND=${ROUND:-r02b} bash scripts/profile_round.sh || exit 1
timeout -k 10 400 python bench.py --workload config5 --steps 2 --warmup 1 --cpu-budget 8 > gpurun_out/bench_${ROUND:-r02b}_config5.json 2> gpurun_out/bench_${ROUND:-r02b}_config5.err || exit 1
cut -c1-300 gpurun_out/bench_${ROUND:-r02b}_config5.json
