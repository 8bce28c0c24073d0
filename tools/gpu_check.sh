#!/bin/bash
# One GPU-box session: parity tests, smoke, a short bench.  Stops at the first step that
# ends in a fault-type status (abort, segfault, time limit) so nothing else touches the GPU.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
fault() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
STEPS="${STEPS:-tests smoke bench}"
for s in $STEPS; do
  case $s in
    tests) timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 180 --timeout-method thread \
             > gpurun_out/gpu_tests.log 2>&1; rc=$? ;;
    smoke) timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" \
             > gpurun_out/smoke.log 2>&1; rc=$? ;;
    bench) timeout -k 10 600 python -u bench.py ${BENCH_ARGS:---steps 2 --warmup 1 --cpu-gens 30} \
             > gpurun_out/bench.json 2> gpurun_out/bench.log; rc=$? ;;
    prof) timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run \
             --output-format csv -- python3 bench.py ${PROF_ARGS:---steps 1 --warmup 0 --no-cpu-baseline --n-gen 200} \
             > gpurun_out/prof.log 2>&1; rc=$? ;;
    *) echo "unknown step $s"; rc=1 ;;
  esac
  echo "step $s rc=$rc"
  if fault $rc; then echo "fault-type exit in $s: stopping"; exit $rc; fi
done
tail -5 gpurun_out/gpu_tests.log 2>/dev/null
cat gpurun_out/smoke.log 2>/dev/null | tail -3
cat gpurun_out/bench.json 2>/dev/null
find gpurun_out/prof -name '*kernel_stats.csv' 2>/dev/null | head -1 | xargs -r head -12
