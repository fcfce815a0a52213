#!/bin/bash
# PMC FETCH_SIZE / WRITE_SIZE passes (KOORDHIP_SERIAL: rocprofv3 --pmc
# serialises dispatches, so no persistent resolve) of the evaluation kernels
# of configs 4 (k_scan) and 5 (k_eval_topk), then bench lines of configs 5 / 4.
set -u
R=${ROUND:-r03d}
KOORDHIP_SERIAL=1 bash scripts/pmc.sh pmc_${R}_config4 --steps 1 --warmup 0 --pods 30000 || exit 1
KOORDHIP_SERIAL=1 bash scripts/pmc.sh pmc_${R}_config5 --workload config5 --steps 1 --warmup 0 --pods 6000 || exit 1
for w in config5 config4; do
  timeout -k 10 300 python bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${R}_$w.json 2> gpurun_out/${R}_$w.err || exit 1
  cut -c1-300 gpurun_out/${R}_$w.json
done
