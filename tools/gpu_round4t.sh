#!/bin/bash
# Phase clocks of the current kernels (MV_CLOCKS build): k_genc, k_mlp2 and survival, one
# state group, botnet headline shape.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/phases; mkdir -p $O
export MOEVA_MI355X_LIB=$PWD/moeva2-ijcai22-replication_amd/lib/libmoeva_mi355x_clk.so
MV_GEN_PHASES=1 timeout -k 10 200 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --n-gen 100 --groups 1 > $O/genc.json 2> $O/genc.log || exit 1
grep "\[mv\] k_genc" $O/genc.log
MV_MLP_PHASES=1 timeout -k 10 200 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --n-gen 100 --groups 1 > $O/mlp.json 2> $O/mlp.log || exit 1
grep "k_mlp phase" $O/mlp.log | tail -1
MV_SURV_PHASES=1 timeout -k 10 200 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --n-gen 100 --groups 1 > $O/surv.json 2> $O/surv.log || exit 1
grep "survival phase" $O/surv.log | tail -1
unset MOEVA_MI355X_LIB
L=$PWD/moeva2-ijcai22-replication_amd/lib
mkdir -p gpurun_out/ab
SETS="MV_MLP2_OCC=2 MOEVA_MI355X_LIB=$L/libmoeva_mi355x_o3.so MOEVA_MI355X_LIB=$L/libmoeva_mi355x_o4.so" REPS=2 STEPS=5 bash tools/gpu_ab_env.sh
