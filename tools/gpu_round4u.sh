#!/bin/bash
# Survival phase split at configs[3] (N = 963, dominance bitsets in HBM), MV_CLOCKS build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/phases; mkdir -p $O
export MOEVA_MI355X_LIB=$PWD/moeva2-ijcai22-replication_amd/lib/libmoeva_mi355x_clk.so
MV_SURV_PHASES=1 timeout -k 10 300 python -u bench.py --workload synthetic.lcld.scaleout --steps 1 --warmup 0 --no-cpu-baseline --n-gen 4 --groups 1 > $O/surv_c4.json 2> $O/surv_c4.log || exit 1
grep "survival phase" $O/surv_c4.log | tail -1
