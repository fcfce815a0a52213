#!/bin/bash
set -u
KOORDHIP_SERIAL=1 bash scripts/pmc_sq.sh sq_c5 --workload config5 --steps 1 --warmup 0 --pods 4000 || exit 1
KOORDHIP_SERIAL=1 bash scripts/pmc_sq.sh sq_c4 --steps 1 --warmup 0 --pods 12000 || exit 1
