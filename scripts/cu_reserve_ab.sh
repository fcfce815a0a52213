KOORDHIP_CU_RESERVE=1 timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_numa.py -x -q --timeout 60 --timeout-method thread > gpurun_out/pt_cu.log 2>&1 && tail -2 gpurun_out/pt_cu.log && \
for G in 7 8; do KOORDHIP_CU_RESERVE=1 KOORDHIP_SEL_G=$G timeout -k 10 120 python bench.py --no-cpu-baseline --steps 3 --warmup 1 | cut -c90-175 || exit 1; done && \
timeout -k 10 120 python bench.py --no-cpu-baseline --steps 3 --warmup 1 | cut -c90-175 && \
KOORDHIP_CU_RESERVE=1 timeout -k 10 120 python bench.py --workload config3 --no-cpu-baseline --steps 3 --warmup 1 | cut -c90-175 && \
timeout -k 10 120 python bench.py --workload config3 --no-cpu-baseline --steps 3 --warmup 1 | cut -c90-175
