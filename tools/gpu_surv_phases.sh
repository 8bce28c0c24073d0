#!/bin/bash
# Survival phase split (MV_SURV_PHASES=1: clock64 cycles of the LAST generation, one state
# group) at several attack lengths on WORKLOAD (default the headline).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/ph; mkdir -p $O
W=${WORKLOAD:-rq1.botnet.static}
for g in ${GENS:-50 300 1000}; do
  MV_SURV_PHASES=1 timeout -k 10 200 python -u bench.py --workload $W --steps 1 --warmup 0 --no-cpu-baseline --n-gen $g --groups 1 > $O/$W.$g.json 2> $O/$W.$g.log || exit 1
  echo "$W n_gen=$g"; grep "\[mv\]" $O/$W.$g.log
done
