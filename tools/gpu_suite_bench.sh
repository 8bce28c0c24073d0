#!/bin/bash
# GPU parity suite (stops at the first failure), then smoke() and the default bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/sb; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $O/gpu_tests.log 2>&1
rc=$?; tail -3 $O/gpu_tests.log; grep -E "^(FAILED|ERROR)" $O/gpu_tests.log | head; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; tail -2 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.log
rc=$?; python3 tools/show_bench.py $O/bench.json; exit $rc
