#!/bin/bash
# node-major scan: parity tests, then scan sweeps on configs 4 / 5 / 3
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/nm_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/nm_pytest.log; [ $rc -eq 0 ] || exit $rc
bash scripts/sweep_scan.sh nm4 config4 "${S4:-2:a 2:0 2:2 2:4 1:a}" || exit 1
bash scripts/sweep_scan.sh nm5 config5 "${S5:-2:a 2:0 1:a 1:4 2:4}" || exit 1
[ -n "${S3:-}" ] && { bash scripts/sweep_scan.sh nm3 config3 "$S3" || exit 1; }
exit 0
