#!/bin/bash
# Classifier phase clocks (clocks build, one state group) for k_mlpr and k_mlp2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/mlprph; mkdir -p $O
export MOEVA_MI355X_LIB=moeva2-ijcai22-replication_amd/lib/libmoeva_mi355x_clk.so
for v in ${VALUES:-1 0}; do
  MV_MLPR=$v MV_MLP_PHASES=1 timeout -k 10 200 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-configs --no-generate --groups 1 --n-gen 50 ${BENCH_ARGS:-} > $O/r$v.json 2> $O/r$v.log || exit 1
  echo "MV_MLPR=$v"; grep "k_mlp phase" $O/r$v.log | tail -1
done
