#!/bin/bash
# One GPU-box pass producing a round's evidence (or a subset of it).
#   ROUND=r04a STAGES="tests smoke bench stamps prof pmc" bash scripts/gpu_round.sh
# stages:
#   tests   full `pytest -m gpu` (TESTS_FILES / TESTS_K narrow it)
#   smoke   __graft_entry__.smoke()
#   bench   bench lines of WORKLOADS (default config4 config3 config5), CPU baseline on
#   quick   bench lines without the CPU baseline (iteration)
#   stamps  KOORDHIP_STAMPS resolve / select cycle stamps per workload
#   prof    rocprofv3 --kernel-trace --stats per workload
#   pmc     FETCH_SIZE / WRITE_SIZE passes per workload (KOORDHIP_SERIAL: no persistent resolve;
#           KOORDHIP_PMC_REPLAY: the class lists' and device pods' launches replayed after each call)
# Every GPU step has its own time limit; the first failure stops the script.
set -u
R=${ROUND:-r04x}
STAGES=${STAGES:-tests smoke bench stamps prof pmc}
WORKLOADS=${WORKLOADS:-config4 config3 config5}
mkdir -p gpurun_out
has() { case " $STAGES " in *" $1 "*) return 0;; esac; return 1; }
steps_of() { case $1 in config4|config4dsmix|config4ds) echo "--steps 5 --warmup 2";; config3|deviceshare|spread|affinity) echo "--steps 3 --warmup 1";; resvpolicy) echo "--steps 1 --warmup 1";; *) echo "--steps 2 --warmup 1";; esac; }
pods_pmc() { case $1 in config4|config4dsmix) echo 100000;; config3) echo 10000;; *) echo 6000;; esac; }

if has tests; then
  FILES=${TESTS_FILES:-tests}
  timeout -k 10 1100 python -u -m pytest $FILES -m gpu -x -q --timeout 300 --timeout-method thread ${TESTS_K:+-k "$TESTS_K"} \
    > gpurun_out/${R}_pytest.log 2>&1
  rc=$?; tail -4 gpurun_out/${R}_pytest.log; [ $rc -eq 0 ] || { tail -40 gpurun_out/${R}_pytest.log; exit $rc; }
fi
if has smoke; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${R}_smoke.log 2>&1 || { cat gpurun_out/${R}_smoke.log; exit 1; }
fi
for w in $WORKLOADS; do
  if has bench || has quick; then
    extra=""; has bench || extra="--no-cpu-baseline"
    timeout -k 10 400 python bench.py --workload $w $(steps_of $w) --cpu-budget 8 $extra ${BENCH_ARGS:-} \
      > gpurun_out/bench_${R}_$w.json 2> gpurun_out/bench_${R}_$w.err || { tail -20 gpurun_out/bench_${R}_$w.err; exit 1; }
    python3 - gpurun_out/bench_${R}_$w.json $w <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
if "eval_roofline" in d:
    print(sys.argv[2], "pods/s", d["value"], "ms/step", d["ms_per_step"], d["eval_roofline"]["kernel"],
          "eval", d["eval_roofline"]["kernel"], d["eval_roofline"].get("avg_launch_us", d["eval_roofline"].get("avg_launch_ms")), "select us", d.get("select", {}).get("avg_launch_us"),
          "P", d["config"]["batch_pods"], "lag", d["config"]["pipeline_lag"], "unsched", d["unschedulable"])
else:  # the sequential cycle's workloads
    print(sys.argv[2], "pods/s", d["value"], "ms/step", d["ms_per_step"], d["roofline"]["kernel"],
          "us/pod", d["roofline"]["us_per_pod"], "unsched", d["unschedulable"])
PY
  fi
  if has stamps; then
    KOORDHIP_STAMPS=1 timeout -k 10 300 python bench.py --workload $w --steps 1 --warmup 1 --no-cpu-baseline --no-latency ${BENCH_ARGS:-} \
      > gpurun_out/stamps_${R}_$w.json 2> gpurun_out/stamps_${R}_$w.err || { tail -20 gpurun_out/stamps_${R}_$w.err; exit 1; }
    grep "stamps\] resolve cycles" gpurun_out/stamps_${R}_$w.err | tail -1 | cut -c1-250
  fi
  if has prof; then
    bash scripts/profile.sh ${R}_$w --workload $w --steps 1 --warmup 1 ${BENCH_ARGS:-} || exit 1
  fi
  if has pmc; then
    KOORDHIP_SERIAL=1 KOORDHIP_PMC_REPLAY=1 bash scripts/pmc.sh pmc_${R}_$w --workload $w --steps 1 --warmup 0 --pods $(pods_pmc $w) ${BENCH_ARGS:-} || exit 1
  fi
done
exit 0
