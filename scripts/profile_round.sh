#!/bin/bash
# One GPU-box pass that produces this round's committed evidence: rocprofv3
# kernel stats of config 4 and config 3, the FETCH_SIZE / WRITE_SIZE passes of
# config 4 (single-stream mode: rocprofv3 --pmc serialises dispatches), and
# the bench lines of both workloads.  Every step is time-limited; the first
# failure stops the script.
set -u
P=${ROUND:-r01c}
bash scripts/profile.sh ${P}_config4 --steps 2 --warmup 1 || exit 1
KOORDHIP_SERIAL=1 bash scripts/pmc.sh pmc_${P} --steps 1 --warmup 0 --pods 30000 || exit 1
timeout -k 10 400 python bench.py --steps 3 --warmup 1 > gpurun_out/bench_${P}.json 2> gpurun_out/bench_${P}.err || exit 1
timeout -k 10 300 python bench.py --workload config3 --steps 3 --warmup 1 --cpu-budget 8 > gpurun_out/bench_${P}_config3.json 2> gpurun_out/bench_${P}_config3.err || exit 1
bash scripts/profile.sh ${P}_config3 --workload config3 --steps 2 --warmup 1 || exit 1
cut -c1-220 gpurun_out/bench_${P}.json gpurun_out/bench_${P}_config3.json
