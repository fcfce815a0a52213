#!/bin/bash
# Resolve A/B: parity selection on each library build, then bench + stamps of config 4.
# Usage: LIBS="base t256" bash scripts/r03_ab.sh
set -u
mkdir -p gpurun_out
for lib in ${LIBS:-base}; do
  if [ "$lib" = base ]; then lp=koordinator_amd/lib/libkoordhip.so; else lp=koordinator_amd/lib/libkoordhip_$lib.so; fi
  KOORDHIP_LIB=$lp timeout -k 10 600 python -u -m pytest ${TESTS_FILES:-tests/test_gpu_parity.py tests/test_gpu_fullsize.py} -m gpu -x -q \
    --timeout 300 --timeout-method thread ${TESTS_K:+-k "$TESTS_K"} > gpurun_out/ab_tests_$lib.log 2>&1
  rc=$?; echo "== $lib tests rc=$rc"; tail -3 gpurun_out/ab_tests_$lib.log; [ $rc -eq 0 ] || exit $rc
  for w in ${WORKLOADS:-config4}; do
    KOORDHIP_LIB=$lp timeout -k 10 300 python bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ab_b_${lib}_$w.json 2>/dev/null || exit 1
    echo "$lib $w $(grep -o '"value": [0-9.]*' gpurun_out/ab_b_${lib}_$w.json | head -1)"
    KOORDHIP_LIB=$lp KOORDHIP_STAMPS=1 timeout -k 10 300 python bench.py --workload $w --steps 1 --warmup 1 --no-cpu-baseline > /dev/null 2> gpurun_out/ab_st_${lib}_$w.err || exit 1
    grep "stamps\] \(resolve\|prologue\|general\|round\)" gpurun_out/ab_st_${lib}_$w.err | cut -c1-300
  done
done
