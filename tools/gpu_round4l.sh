#!/bin/bash
# k_mlp2 two-set layer-0 pipeline: GPU suite (f1 bit-exact in engine order), headline A/B
# against the previous library (prev), k_mlp2 phase clocks not needed.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r4
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r4/suite_mlp2set.log 2>&1
rc=$?; tail -n 2 gpurun_out/r4/suite_mlp2set.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error" gpurun_out/r4/suite_mlp2set.log | head; exit $rc; }
L=$PWD/moeva2-ijcai22-replication_amd/lib
SETS="MV_SLIM=1 MOEVA_MI355X_LIB=$L/libmoeva_mi355x_prev.so" REPS=2 STEPS=6 bash tools/gpu_ab_env.sh
