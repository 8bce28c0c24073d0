#!/bin/bash
# Quick perf check: per-kernel split with one state group, then the default bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
timeout -k 10 200 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --n-gen 200 --groups 1 \
  > gpurun_out/ab/g1.json 2> gpurun_out/ab/g1.log || exit $?
echo "groups=1 $(python3 tools/show_bench.py gpurun_out/ab/g1.json | head -1)"
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline \
  > gpurun_out/ab/def.json 2> gpurun_out/ab/def.log || exit $?
echo "default $(python3 tools/show_bench.py gpurun_out/ab/def.json | head -1)"
