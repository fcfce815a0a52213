#!/bin/bash
# SQ instruction / stall counters of a short bench run (one rocprofv3 --pmc pass
# per group; <= 8 SQ counters per pass).  Usage: scripts/pmc_sq.sh NAME [bench args...]
set -u
name=$1; shift
export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM"; do
  i=$((i+1))
  mkdir -p gpurun_out/$name/g$i
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/$name/g$i -o run \
    -- python3 bench.py --no-cpu-baseline "$@" > gpurun_out/$name/g$i/bench.log 2>&1 || { echo "pmc group $i failed rc=$?"; tail -5 gpurun_out/$name/g$i/bench.log; exit 1; }
done
echo "pmc ok" >&2
