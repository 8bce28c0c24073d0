#!/bin/bash
# bf16 perf mode round: its GPU tests, then fp32 vs bf16 bench lines on the headline
# (rq1.botnet.static) and the wide-MLP config (synthetic.botnet.wide).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/bf16
mkdir -p $O
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "bf16 or wide" -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -4 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for W in rq1.botnet.static synthetic.botnet.wide; do
  for D in fp32 bf16; do
    timeout -k 10 300 python -u bench.py --workload $W --mlp-dtype $D --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_${W}_$D.json 2> $O/bench_${W}_$D.log || exit $?
    python3 tools/show_bench.py $O/bench_${W}_$D.json
  done
done
