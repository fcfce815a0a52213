#!/bin/bash
# k_scan pods-per-wave / nodes-per-lane sweep (bench only).
# Usage: scripts/sweep_scan.sh OUTDIR WORKLOAD "R:PPW ..."   (PPW a = automatic node-major, 0 = pod-major k_scan)
set -u
out=gpurun_out/${1:-scan_sweep}
w=${2:-config4}
mkdir -p $out
for rp in ${3:-"2:a 2:0 1:a 2:4 2:8"}; do
  r=${rp%%:*}; ppw=${rp##*:}
  tag=${w}_r${r}_p${ppw}
  if [ $ppw = a ]; then export KOORDHIP_SCAN_PPW=auto; else export KOORDHIP_SCAN_PPW=$ppw; fi
  KOORDHIP_TOPK_R=$r timeout -k 10 300 python bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline \
    > $out/$tag.json 2> $out/$tag.err || { echo "failed $tag"; exit 1; }
  python - "$out/$tag.json" "$tag" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(sys.argv[2], d["value"], d["eval_roofline"]["avg_launch_us"], d["select"]["avg_launch_us"], flush=True)
PY
done
