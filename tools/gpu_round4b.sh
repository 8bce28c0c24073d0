#!/bin/bash
# Round 4: GPU suite (default library), survival duplicate hunt (checks build), headline
# bench + rocprofv3 kernel stats of the same command.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r4
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests \
  -k "not test_success_rate_within_1pp_state_streams or lcld" > gpurun_out/r4/suite.log 2>&1
rc=$?
tail -n 4 gpurun_out/r4/suite.log
[ $rc -ne 0 ] && exit $rc
bash tools/gpu_surv_dump.sh || exit $?
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r4/bench.json 2> gpurun_out/r4/bench.log || exit $?
cat gpurun_out/r4/bench.json
