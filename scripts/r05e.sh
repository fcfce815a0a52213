#!/bin/bash
# full GPU suite + smoke on the current build
set -u
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05e_pytest.log 2>&1
rc=$?; tail -4 gpurun_out/r05e_pytest.log; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error" gpurun_out/r05e_pytest.log | head -20; tail -60 gpurun_out/r05e_pytest.log; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05e_smoke.log 2>&1 || { cat gpurun_out/r05e_smoke.log; exit 1; }
tail -2 gpurun_out/r05e_smoke.log
