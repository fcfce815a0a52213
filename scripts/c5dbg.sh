set -u
for v in "KOORDHIP_TOPK_R=1 KOORDHIP_ROUND_LAUNCH=1" "KOORDHIP_TOPK_R=1 KOORDHIP_SERIAL=1" "KOORDHIP_TOPK_R=1 KOORDHIP_SELECT_ONEWG=1" "KOORDHIP_TOPK_R=2"; do
  echo "== $v"
  env $v timeout -k 10 200 python bench.py --workload config5 --nodes 200000 --pods 2000 --steps 1 --warmup 0 --no-cpu-baseline 2>&1 | grep -v amdgpu.ids | cut -c1-250 | tail -2
done
