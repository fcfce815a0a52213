set -u
true
KOORDHIP_SERIAL=1 bash scripts/pmc.sh pmc_r01c --steps 1 --warmup 0 --pods 30000 || exit 1
timeout -k 10 400 python bench.py --steps 3 --warmup 1 > gpurun_out/bench_r01c.json 2> gpurun_out/bench_r01c.err || exit 1
timeout -k 10 300 python bench.py --workload config3 --steps 3 --warmup 1 --cpu-budget 8 > gpurun_out/bench_r01c_config3.json 2> gpurun_out/bench_r01c_config3.err || exit 1
bash scripts/profile.sh r01c_config3 --workload config3 --steps 2 --warmup 1 || exit 1
cut -c1-220 gpurun_out/bench_r01c.json gpurun_out/bench_r01c_config3.json
