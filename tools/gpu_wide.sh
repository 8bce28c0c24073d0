#!/bin/bash
# Wide-MLP (configs[4]) bf16 round: the bf16 / wide GPU tests, then the wide workload's bench
# lines (bf16 and fp32) and a rocprofv3 kernel-stats pass of the bf16 line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/wide
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "bf16 or wide or sharded" -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -6 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for D in bf16 fp32; do
  timeout -k 10 300 python -u bench.py --workload synthetic.botnet.wide --mlp-dtype $D --steps 2 --warmup 1 > $O/bench_$D.json 2> $O/bench_$D.log || exit $?
  python3 tools/show_bench.py $O/bench_$D.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --workload synthetic.botnet.wide --mlp-dtype bf16 --steps 1 --warmup 1 --groups 1 --n-gen 20 > $O/prof.log 2>&1 || exit $?
cp $(find $O/prof -name '*kernel_stats.csv' | head -1) $O/kernel_stats_bf16.csv; head -6 $O/kernel_stats_bf16.csv
