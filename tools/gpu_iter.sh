#!/bin/bash
# One iteration on a GPU box: the GPU parity suite (stops at the first failure; PYTEST_K
# narrows it), then an A/B of the headline bench between library builds / env sets
# (SETS, as tools/gpu_ab_env.sh; skipped when empty), then (PHASES=1) the phase clocks.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/it; mkdir -p $O
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $O/gpu_tests.log 2>&1
  rc=$?; tail -3 $O/gpu_tests.log; grep -E "^(FAILED|ERROR)" $O/gpu_tests.log | head; [ $rc -eq 0 ] || exit $rc
fi
[ -n "$SETS" ] && { SETS="$SETS" REPS=${REPS:-2} STEPS=${STEPS:-4} bash tools/gpu_ab_env.sh || exit 1; }
# PHASES=1: k_genc and survival phase clocks with the clocks build (make variant NAME=clk)
if [ -n "$PHASES" ]; then
  export MOEVA_MI355X_LIB=$PWD/moeva2-ijcai22-replication_amd/lib/libmoeva_mi355x_clk.so
  ROWS=32 GENS=100 bash tools/gpu_genc_phases.sh || exit 1
  GENS="50 1000" bash tools/gpu_surv_phases.sh || exit 1
fi
exit 0
