#!/bin/bash
# Survival-kernel iteration on one GPU box: GPU parity tests, survival phase split
# (MV_SURV_PHASES=1), headline bench line.  Stops at the first failing step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/surv
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
MV_SURV_PHASES=1 timeout -k 10 120 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --n-gen 50 --groups 1 > $O/phases.json 2> $O/phases.log || exit 1
grep "\[mv\]" $O/phases.log
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.log || exit 1
python3 tools/show_bench.py $O/bench.json
