#!/bin/bash
# Round measurement on one GPU box: parity tests, rocprofv3 kernel stats of the bench,
# two PMC passes (FETCH_SIZE, WRITE_SIZE) -> profiles/pmc_traffic.json, then the bench
# line (which reads that traffic).  Stops at the first fault-type exit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/round
O=gpurun_out/round
fault() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
run() { local name=$1; shift; "$@"; local rc=$?; echo "step $name rc=$rc"; if fault $rc; then echo "fault-type exit in $name"; exit $rc; fi; return 0; }
STEPS="${STEPS:-tests prof pmc bench}"
for s in $STEPS; do
  case $s in
    tests) run tests timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 180 --timeout-method thread > $O/gpu_tests.log 2>&1
           tail -3 $O/gpu_tests.log ;;
    prof) run prof timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --groups 1 > $O/prof.log 2>&1
          cp $(find $O/prof -name '*kernel_stats.csv' | head -1) $O/kernel_stats.csv ;;
    pmc) run pmc_fetch timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --n-gen 20 --groups 1 > $O/pmc_fetch.log 2>&1
         run pmc_write timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmc_write -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --n-gen 20 --groups 1 > $O/pmc_write.log 2>&1
         python3 tools/pmc_traffic.py profiles/pmc_traffic.json $(find $O/pmc_fetch $O/pmc_write -name '*counter_collection.csv') > $O/pmc_traffic.log 2>&1
         cp profiles/pmc_traffic.json $O/ ; cat $O/pmc_traffic.log ;;
    bench) run bench bash -c "timeout -k 10 600 python -u bench.py ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.log"
           python3 tools/show_bench.py $O/bench.json ;;
  esac
done
find $O/prof -name '*kernel_stats.csv' | head -1 | xargs -r head -12
