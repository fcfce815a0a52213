#!/bin/bash
# Focused GPU check (FILES, default the reservation files), then optionally
# the round evidence (ROUND set: scripts/gpu_round.sh).  Each GPU step is
# time-limited; the first failure stops the script.
set -u
mkdir -p gpurun_out
FILES=${FILES:-"tests/test_resv_cpus.py tests/test_reservation_slots.py tests/test_gpu_reservation.py"}
timeout -k 10 600 python -u -m pytest $FILES -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/check.log 2>&1
rc=$?; tail -30 gpurun_out/check.log; [ $rc -eq 0 ] || exit $rc
if [ -n "${ROUND:-}" ]; then bash scripts/gpu_round.sh; fi
