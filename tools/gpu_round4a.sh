#!/bin/bash
# Survival duplicate hunt (checks build) + the default library's GPU suite.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/fault
bash tools/gpu_surv_dump.sh || exit $?
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests \
  -k "not test_success_rate_within_1pp_state_streams or lcld" > gpurun_out/fault/suite4.log 2>&1
rc=$?
tail -n 5 gpurun_out/fault/suite4.log
exit $rc
