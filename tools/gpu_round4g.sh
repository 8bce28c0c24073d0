#!/bin/bash
# Slim k_genc phase-2 LDS: bit-identity + GPU suite, then the headline A/B: slim (default)
# vs full region A (MV_SLIM=0) vs slim with k_genc at 4 waves/SIMD (the w4 library).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r4
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests \
  -k "not test_success_rate_within_1pp_state_streams or lcld" > gpurun_out/r4/suite_slim.log 2>&1
rc=$?; tail -n 3 gpurun_out/r4/suite_slim.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error" gpurun_out/r4/suite_slim.log | head; exit $rc; }
L=$PWD/moeva2-ijcai22-replication_amd/lib
SETS="MV_SLIM=1 MV_SLIM=0 MOEVA_MI355X_LIB=$L/libmoeva_mi355x_w4.so" REPS=2 STEPS=6 bash tools/gpu_ab_env.sh
