#!/bin/bash
# Round-4 final measurement: smoke(), then tools/gpu_round.sh (GPU suite, rocprofv3 kernel
# stats, timeline, PMC traffic / MFMA passes, bench line) with ROUND=r04.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/final
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1
rc=$?; tail -n 2 gpurun_out/final/smoke.log; [ $rc -ne 0 ] && exit $rc
ROUND=r04 bash tools/gpu_round.sh
