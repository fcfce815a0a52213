#!/bin/bash
# One GPU-box pass: parity tests, smoke, short bench.  Each GPU step has its
# own time limit; a crash/abort/timeout (exit status other than 0/1) stops the
# script so nothing else runs on a possibly faulted GPU.
set -u
mkdir -p gpurun_out
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name" >&2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" >&2
  tail -5 "gpurun_out/$name.log" >&2
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)" >&2; exit $rc; fi
  return $rc
}
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench 600 python bench.py --steps ${BENCH_STEPS:-2} --warmup 1 --cpu-budget ${CPU_BUDGET:-8}
exit 0
