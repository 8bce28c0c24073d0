#!/bin/bash
# GPU parity suite (all tests, no -x) with per-test timeout; PYTEST_K (a -k expression) narrows it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} \
  > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests.log; grep -E "^(FAILED|ERROR)" gpurun_out/gpu_tests.log | head -20
exit $rc
