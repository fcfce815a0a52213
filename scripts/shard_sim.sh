#!/bin/bash
# The expected node-shard curve on one GPU:
# KOORDHIP_SHARD_SIM=W makes a one-rank context evaluate only shard 0 of W
# through the full exchange path (--one-rank-comm), W = 1 2 4 8, per workload.
# Timing only (the placements of a simulated shard differ).
set -u
mkdir -p gpurun_out
for wl in ${WORKLOADS:-config4 config5}; do
  for w in 1 2 4 8; do
    KOORDHIP_SHARD_SIM=$w timeout -k 10 300 python bench.py --workload $wl --one-rank-comm --steps ${STEPS:-3} --warmup 1 \
      --no-cpu-baseline --no-latency > gpurun_out/shardsim_${wl}_$w.json 2> gpurun_out/shardsim_${wl}_$w.err || { tail -5 gpurun_out/shardsim_${wl}_$w.err; exit 1; }
    python3 - gpurun_out/shardsim_${wl}_$w.json $wl $w <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
e = d["eval_roofline"]
print(sys.argv[2], "W", sys.argv[3], "pods/s", d["value"], "ms/step", d["ms_per_step"], e["kernel"],
      "eval us", e.get("avg_launch_us"), "select us", d.get("select", {}).get("avg_launch_us"))
PY
  done
done
