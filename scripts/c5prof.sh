cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for w in 2 4 8; do
  KOORDHIP_SHARD_SIM=$w timeout -k 10 300 python bench.py --workload config5 --steps 2 --warmup 1 --no-cpu-baseline --one-rank-comm > gpurun_out/sim5_$w.json 2> gpurun_out/sim5_$w.err || exit 1
  KOORDHIP_SHARD_SIM=$w timeout -k 10 300 python bench.py --workload config4 --steps 2 --warmup 1 --no-cpu-baseline --one-rank-comm > gpurun_out/sim4_$w.json 2> gpurun_out/sim4_$w.err || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5x -o run -- python3 bench.py --workload config5 --steps 1 --warmup 0 --no-cpu-baseline --one-rank-comm > gpurun_out/prof_c5x.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5 -o run -- python3 bench.py --workload config5 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/prof_c5.log 2>&1
