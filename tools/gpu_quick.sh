#!/bin/bash
# Quick GPU iteration: parity tests then a short bench (kernel split per generation).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread \
  > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests.log; grep -E "^(FAILED|E )" gpurun_out/gpu_tests.log | head -20
case $rc in 124|134|137|139) echo "fault-type exit $rc"; exit $rc;; esac
timeout -k 10 300 python -u bench.py ${BENCH_ARGS:---steps 1 --warmup 1 --no-cpu-baseline --n-gen 200} \
  > gpurun_out/bench.json 2> gpurun_out/bench.log || exit 1
python3 tools/show_bench.py gpurun_out/bench.json
