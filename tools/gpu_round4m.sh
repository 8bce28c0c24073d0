#!/bin/bash
# Compact gene layout: GPU suite, then the headline A/B (compact vs MV_COMPACT=0) and the
# SBX option A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r4
rm -f gpurun_out/ab/*
timeout -k 10 800 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests --deselect "tests/test_gpu_e2e.py::test_success_rate_within_1pp_at_full_config[e2e_botnet_rq1.npz]" > gpurun_out/r4/suite_compact.log 2>&1
rc=$?; tail -n 3 gpurun_out/r4/suite_compact.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/r4/suite_compact.log | head -30; exit $rc; }
SETS="MV_COMPACT=1 MV_COMPACT=0" REPS=2 STEPS=6 bash tools/gpu_ab_env.sh || exit 1
SETS="MV_COMPACT=1 MV_COMPACT=0" REPS=1 STEPS=3 BENCH_ARGS="--crossover sbx" bash tools/gpu_ab_env.sh
