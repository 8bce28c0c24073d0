#!/bin/bash
# det_pow with FMA exact products (bit-identical): GPU suite, then the headline and the SBX
# option (default 3-wave SBX instance vs a 4-wave variant).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r4 gpurun_out/ab
timeout -k 10 800 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests --deselect "tests/test_gpu_e2e.py::test_success_rate_within_1pp_at_full_config[e2e_botnet_rq1.npz]" > gpurun_out/r4/suite_fma.log 2>&1
rc=$?; tail -n 3 gpurun_out/r4/suite_fma.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/r4/suite_fma.log | head -30; exit $rc; }
L=$PWD/moeva2-ijcai22-replication_amd/lib
SETS="MV_COMPACT=1" REPS=2 STEPS=6 bash tools/gpu_ab_env.sh || exit 1
SETS="MV_SBX=3 MOEVA_MI355X_LIB=$L/libmoeva_mi355x_sbx4.so" REPS=2 STEPS=3 BENCH_ARGS="--crossover sbx" bash tools/gpu_ab_env.sh
