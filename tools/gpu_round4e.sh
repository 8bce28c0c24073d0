#!/bin/bash
# k_mlp2 8-wave tiles: bit-identity tests, then the headline A/B against 4-wave tiles.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r4
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_parity.py -k "eight_wave" > gpurun_out/r4/mlp8.log 2>&1
rc=$?; tail -n 3 gpurun_out/r4/mlp8.log; [ $rc -ne 0 ] && exit $rc
SETS="MV_MLP_WAVES=4 MV_MLP_WAVES=8" REPS=2 STEPS=6 bash tools/gpu_ab_env.sh
