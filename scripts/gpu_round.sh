#!/bin/bash
# Round evidence: full GPU suite + smoke, bench lines of configs 4 / 3 / 5, rocprofv3 kernel stats of configs 3, 4 and 5.
# Usage: ROUND=r02x bash scripts/gpu_round.sh (through scripts/gpu.sh)
set -u
R=${ROUND:-r02c}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${R}_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/${R}_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${R}_smoke.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/bench_${R}.json 2> gpurun_out/bench_${R}.err || exit 1
timeout -k 10 300 python bench.py --workload config3 --steps 3 --warmup 1 --cpu-budget 8 > gpurun_out/bench_${R}_config3.json 2> gpurun_out/bench_${R}_config3.err || exit 1
timeout -k 10 400 python bench.py --workload config5 --steps 2 --warmup 1 --cpu-budget 8 > gpurun_out/bench_${R}_config5.json 2> gpurun_out/bench_${R}_config5.err || exit 1
bash scripts/profile.sh ${R}_config3 --workload config3 --steps 2 --warmup 1 || exit 1
bash scripts/profile.sh ${R}_config4 --steps 2 --warmup 1 || exit 1
bash scripts/profile.sh ${R}_config5 --workload config5 --steps 1 --warmup 1 || exit 1
for f in bench_${R} bench_${R}_config3 bench_${R}_config5; do cut -c1-200 gpurun_out/$f.json; done
