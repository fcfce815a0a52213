#!/bin/bash
# rocprofv3 kernel-trace + stats of a bench run (no PMC here; counters are a
# separate pass, see scripts/pmc.sh).  Usage: scripts/profile.sh NAME [bench args...]
set -u
name=$1; shift
export TMPDIR=/tmp
mkdir -p gpurun_out/$name
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$name -o run \
  -- python3 bench.py --no-cpu-baseline "$@" > gpurun_out/$name/bench.log 2>&1
rc=$?
echo "profile rc=$rc" >&2
find gpurun_out/$name -name "*stats*" | head >&2
exit $rc
