#!/bin/bash
# Phase clocks of k_genc, k_mlp2 and k_survive (MV_CLOCKS build), one state group, generation 50.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r4
L=$PWD/moeva2-ijcai22-replication_amd/lib/libmoeva_mi355x_clk.so
for v in MV_GEN_PHASES MV_MLP_PHASES MV_SURV_PHASES; do
  env MOEVA_MI355X_LIB=$L $v=1 timeout -k 10 200 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --n-gen 50 --groups 1 \
    > gpurun_out/r4/ph_$v.json 2> gpurun_out/r4/ph_$v.log || exit 1
  echo "$v:"; grep "\[mv\]" gpurun_out/r4/ph_$v.log
done
