#!/bin/bash
# Survival workgroups of 256 threads (MV_SURV_T=256 variant): survival + attack GPU tests with
# that library, then the headline A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r4 gpurun_out/ab
L=$PWD/moeva2-ijcai22-replication_amd/lib
MOEVA_MI355X_LIB=$L/libmoeva_mi355x_s256.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "survival or tournament or attack_chain or compact or state_groups or population_640" > gpurun_out/r4/suite_s256.log 2>&1
rc=$?; tail -n 3 gpurun_out/r4/suite_s256.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/r4/suite_s256.log | head -30; exit $rc; }
SETS="MV_SURV=512 MOEVA_MI355X_LIB=$L/libmoeva_mi355x_s256.so" REPS=2 STEPS=6 bash tools/gpu_ab_env.sh || exit 1
SETS="MV_SURV=512 MOEVA_MI355X_LIB=$L/libmoeva_mi355x_s256.so" REPS=1 STEPS=1 BENCH_ARGS="--workload synthetic.lcld.scaleout --warmup 1" bash tools/gpu_ab_env.sh
