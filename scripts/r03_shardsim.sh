#!/bin/bash
# Expected multi-GPU curve: KOORDHIP_SHARD_SIM=W through the one-rank RCCL
# exchange path (rank 0's shard of W; placements differ, timing only).
set -u
mkdir -p gpurun_out
for w in config5 config4; do
  for W in 1 2 4 8; do
    KOORDHIP_SHARD_SIM=$W timeout -k 10 300 python bench.py --workload $w --one-rank-comm --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ss_${w}_$W.json 2> gpurun_out/ss_${w}_$W.err || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['eval_roofline']['avg_launch_us'], d['select']['avg_launch_us'], d['config']['batch_pods'], d['config']['pipeline_lag'])" gpurun_out/ss_${w}_$W.json "$w W=$W"
  done
done
