#!/bin/bash
# Slim phase 2 with SlotRow operands (row buffer = the stored mutable features only):
# GPU suite, then the headline A/B against HEAD's full-row build and the 5-waves variant.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r4 gpurun_out/ab
timeout -k 10 800 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r4/suite_slotrow.log 2>&1
rc=$?; tail -n 3 gpurun_out/r4/suite_slotrow.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/r4/suite_slotrow.log | head -30; exit $rc; }
L=$PWD/moeva2-ijcai22-replication_amd/lib
SETS="MV_SLOTROW=1 MOEVA_MI355X_LIB=$L/libmoeva_mi355x_fullrow.so MOEVA_MI355X_LIB=$L/libmoeva_mi355x_w5.so" REPS=2 STEPS=6 bash tools/gpu_ab_env.sh
