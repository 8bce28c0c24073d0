#!/bin/bash
# Parallel mutation draws in row_draws: GPU suite, headline + SBX A/B against the previous library.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r4 gpurun_out/ab
timeout -k 10 800 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r4/suite_pdraws.log 2>&1
rc=$?; tail -n 3 gpurun_out/r4/suite_pdraws.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/r4/suite_pdraws.log | head -30; exit $rc; }
L=$PWD/moeva2-ijcai22-replication_amd/lib
SETS="MV_PDRAWS=1 MOEVA_MI355X_LIB=$L/libmoeva_mi355x_prev.so" REPS=2 STEPS=6 bash tools/gpu_ab_env.sh || exit 1
SETS="MV_PDRAWS=1 MOEVA_MI355X_LIB=$L/libmoeva_mi355x_prev.so" REPS=1 STEPS=3 BENCH_ARGS="--crossover sbx" bash tools/gpu_ab_env.sh
