#!/bin/bash
# Niching member ranks by bitonic sort for long last fronts: survival / attack GPU tests,
# then configs[3] (N = 963) and the headline against the previous library.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r4 gpurun_out/ab
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "survival or tournament or attack or compact or population_640" > gpurun_out/r4/suite_nsort.log 2>&1
rc=$?; tail -n 3 gpurun_out/r4/suite_nsort.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/r4/suite_nsort.log | head -30; exit $rc; }
L=$PWD/moeva2-ijcai22-replication_amd/lib
SETS="MV_NSORT=1 MOEVA_MI355X_LIB=$L/libmoeva_mi355x_prev.so" REPS=2 STEPS=1 BENCH_ARGS="--workload synthetic.lcld.scaleout --warmup 1" bash tools/gpu_ab_env.sh || exit 1
SETS="MV_NSORT=1 MOEVA_MI355X_LIB=$L/libmoeva_mi355x_prev.so" REPS=1 STEPS=5 bash tools/gpu_ab_env.sh
