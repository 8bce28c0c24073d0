#!/bin/bash
# Survival iteration: the survival / attack GPU parity tests, then the survival phase split
# (MV_SURV_PHASES=1, clock64 cycles at generation 50) on the headline and the scale-out
# workloads, then the headline bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/ph; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for w in rq1.botnet.static synthetic.lcld.scaleout; do
  MV_SURV_PHASES=1 timeout -k 10 200 python -u bench.py --workload $w --steps 1 --warmup 0 --no-cpu-baseline --n-gen 50 --groups 1 > $O/$w.json 2> $O/$w.log || exit 1
  echo $w; grep "\[mv\]" $O/$w.log
done
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.log || exit 1
python3 tools/show_bench.py $O/bench.json
