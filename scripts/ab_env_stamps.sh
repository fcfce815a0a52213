set -u
mkdir -p gpurun_out
for v in KOORDHIP_NO_KEY_TABLES=1 KOORDHIP_NO_PRELOAD=1 X=1; do
  env $v KOORDHIP_STAMPS=1 timeout -k 10 300 python bench.py --workload config4 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/st_$v.json 2> gpurun_out/st_$v.err || exit 1
  echo "== $v"; grep stamps gpurun_out/st_$v.err | tail -6 | cut -c1-330
  env $v timeout -k 10 300 python bench.py --workload config4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/b_$v.json 2>/dev/null || exit 1
  cut -c1-260 gpurun_out/b_$v.json | grep -o '"value": [0-9.]*'
done
