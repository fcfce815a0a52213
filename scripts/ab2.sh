#!/bin/bash
# A/B of pipeline knobs at the current defaults (bench only, each run time-limited).
set -u
b() { timeout -k 10 120 python bench.py --no-cpu-baseline --steps 3 --warmup 1 "$@" | cut -c90-150; }
echo "config4 default";   b || exit 1
echo "config4 fold-wait"; KOORDHIP_FOLD_WAIT=1 b || exit 1
echo "config4 default";   b || exit 1
for R in 1 2 4; do echo "config3 R=$R"; KOORDHIP_TOPK_R=$R b --workload config3 || exit 1; done
