#!/bin/bash
# SBX headline: k_genc's SBX instance at 3 waves/SIMD (sbx3 library) vs the allocator's 2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r4
L=$PWD/moeva2-ijcai22-replication_amd/lib
MOEVA_MI355X_LIB=$L/libmoeva_mi355x_sbx3.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_parity.py -k "sbx" > gpurun_out/r4/sbx3_tests.log 2>&1
rc=$?; tail -n 2 gpurun_out/r4/sbx3_tests.log; [ $rc -ne 0 ] && exit $rc
SETS="MV_SLIM=1 MOEVA_MI355X_LIB=$L/libmoeva_mi355x_sbx3.so" REPS=2 STEPS=4 BENCH_ARGS="--crossover sbx" bash tools/gpu_ab_env.sh
timeout -k 10 400 python -u -m pytest -s -q --timeout 300 --timeout-method thread tests/test_gpu_e2e.py \
  -k "state_streams or distribution" > gpurun_out/r4/e2e_print.log 2>&1
grep -A8 "oracle seeds" gpurun_out/r4/e2e_print.log
