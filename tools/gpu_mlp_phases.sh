#!/bin/bash
# Classifier phase clocks (MV_MLP_PHASES, profiled single-group run) per MV_MLPX value.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/mlpph; mkdir -p $O
for v in ${VALUES:-1 0}; do
  MV_MLPX=$v MV_MLP_PHASES=1 timeout -k 10 200 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > $O/x$v.json 2> $O/x$v.log || exit 1
  echo "MV_MLPX=$v"; grep "k_mlp phase" $O/x$v.log | tail -2
done
