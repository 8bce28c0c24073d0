#!/bin/bash
# Association with 4 lanes per individual when more than T/2 are ranked: GPU suite, then the
# headline and configs[3] against the previous library.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r4 gpurun_out/ab
timeout -k 10 800 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r4/suite_assoc4.log 2>&1
rc=$?; tail -n 3 gpurun_out/r4/suite_assoc4.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/r4/suite_assoc4.log | head -30; exit $rc; }
L=$PWD/moeva2-ijcai22-replication_amd/lib
SETS="MV_ASSOC4=1 MOEVA_MI355X_LIB=$L/libmoeva_mi355x_prev.so" REPS=2 STEPS=6 bash tools/gpu_ab_env.sh || exit 1
SETS="MV_ASSOC4=1 MOEVA_MI355X_LIB=$L/libmoeva_mi355x_prev.so" REPS=1 STEPS=1 BENCH_ARGS="--workload synthetic.lcld.scaleout --warmup 1" bash tools/gpu_ab_env.sh
