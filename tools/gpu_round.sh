#!/bin/bash
# Round measurement on one GPU box: parity tests, rocprofv3 kernel stats of the bench (one
# state group, so every launch covers all states), a kernel-trace timeline with the bench's
# default groups, PMC passes (FETCH_SIZE, WRITE_SIZE -> traffic; MFMA busy) and the bench
# line.  WORKLOAD / MODE select the bench workload and schedule.  Stops at the first
# fault-type exit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
W="${WORKLOAD:-rq1.botnet.static}"
M="${MODE:-chain}"
O=gpurun_out/round/$W.$M
mkdir -p $O
BA="--workload $W --mode $M"
fault() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
run() { local name=$1; shift; "$@"; local rc=$?; echo "step $name rc=$rc"; if fault $rc; then echo "fault-type exit in $name"; exit $rc; fi; return 0; }
STEPS="${STEPS:-tests prof timeline pmc bench}"
for s in $STEPS; do
  case $s in
    tests) run tests timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread > $O/gpu_tests.log 2>&1
           tail -3 $O/gpu_tests.log ;;
    prof) run prof timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py $BA --steps 2 --warmup 1 --no-cpu-baseline --no-generate --groups 1 > $O/prof.log 2>&1
          cp $(find $O/prof -name '*kernel_stats.csv' | head -1) $O/kernel_stats.csv ;;
    timeline) run timeline timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tl -o run --output-format csv -- python3 bench.py $BA --steps 1 --warmup 1 --no-cpu-baseline --no-generate --no-configs --n-gen 200 > $O/tl.log 2>&1
          python3 tools/timeline.py $(find $O/tl -name '*kernel_trace.csv' | head -1) > $O/timeline.txt 2>&1; cat $O/timeline.txt ;;
    pmc) run pmc_fetch timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc_fetch -o run --output-format csv -- python3 bench.py $BA --steps 1 --warmup 0 --no-cpu-baseline --n-gen 20 --groups 1 > $O/pmc_fetch.log 2>&1
         run pmc_write timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmc_write -o run --output-format csv -- python3 bench.py $BA --steps 1 --warmup 0 --no-cpu-baseline --n-gen 20 --groups 1 > $O/pmc_write.log 2>&1
         run pmc_mfma timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $O/pmc_mfma -o run --output-format csv -- python3 bench.py $BA --steps 1 --warmup 0 --no-cpu-baseline --n-gen 20 --groups 1 > $O/pmc_mfma.log 2>&1
         mkdir -p profiles/${ROUND:-r03}
         python3 tools/pmc_traffic.py profiles/${ROUND:-r03}/pmc_traffic_${W}_${M}.json $(find $O/pmc_fetch $O/pmc_write -name '*counter_collection.csv') > $O/pmc_traffic.log 2>&1
         python3 tools/pmc_summary.py $(find $O/pmc_mfma -name '*counter_collection.csv') > $O/pmc_mfma.txt 2>&1
         cp profiles/${ROUND:-r03}/pmc_traffic_${W}_${M}.json $O/ ; cat $O/pmc_traffic.log $O/pmc_mfma.txt ;;
    bench) run bench bash -c "timeout -k 10 600 python -u bench.py $BA ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.log"
           python3 tools/show_bench.py $O/bench.json ;;
  esac
done
find $O/prof -name '*kernel_stats.csv' 2>/dev/null | head -1 | xargs -r head -12
