#!/bin/bash
# k_mlpr bring-up: the whole parity suite (failures reported, the A/B still runs unless the
# run crashed), then the headline A/B of the classifier kernels (tools/gpu_ab_env.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/mlpr; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $O/gpu_tests.log 2>&1
rc=$?; echo "tests: $(tail -1 $O/gpu_tests.log)"
[ $rc -eq 0 ] || grep -E "^(FAILED|ERROR)|Error|assert" $O/gpu_tests.log | head -20
[ $rc -le 1 ] || exit $rc
SETS="${SETS:-MV_MLPR=0 MV_MLPR=1 MV_MLPR_RW=1}" REPS=${REPS:-2} STEPS=${STEPS:-4} bash tools/gpu_ab_env.sh || exit 1
exit $rc
