#!/bin/bash
# Round-end measurement on one GPU box: the GPU parity suite, smoke(), the default bench line
# (headline + every BASELINE config + CPU baseline), then a rocprofv3 kernel-trace --stats
# pass of the headline with one state group (its per-kernel averages compare 1:1 with the
# bench line's event-timed roofline pass).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/final; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -2 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; tail -1 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.log
rc=$?; python3 tools/show_bench.py $O/bench.json; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
  python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-configs --groups 1 > $O/prof_bench.json 2> $O/prof_bench.log
rc=$?; echo "rocprof rc=$rc"; exit $rc
