#!/bin/bash
# k_genc at 4 waves/SIMD (128 VGPRs, the w4 library) with the slim phase-2 LDS: headline A/B
# against the default library (3 waves/SIMD) and against w4 with the full region A.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r4
L=$PWD/moeva2-ijcai22-replication_amd/lib
SETS="MOEVA_MI355X_LIB=$L/libmoeva_mi355x_w4.so MV_SLIM=1 MOEVA_MI355X_LIB=$L/libmoeva_mi355x_w4.so,MV_SLIM=0" REPS=2 STEPS=6 bash tools/gpu_ab_env.sh
