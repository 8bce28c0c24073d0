#!/bin/bash
# Library variants on one GPU box: the parity subset PYTEST_K with each library of LIBS
# (names: "" = the product build, else lib/libmoeva_mi355x_<name>.so), stopping at the first
# failure; then the headline A/B over the same libraries (tools/gpu_ab_env.sh); then
# (PHASES=1) the phase clocks of the clocks build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/libs; mkdir -p $O
L=moeva2-ijcai22-replication_amd/lib
path() { [ -z "$1" -o "$1" = main ] && echo $L/libmoeva_mi355x.so || echo $L/libmoeva_mi355x_$1.so; }
K="${PYTEST_K:-survival or attack or compact or slim or evaluate or variation}"
for n in ${TEST_LIBS:-$LIBS}; do
  MOEVA_MI355X_LIB=$(path $n) timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > $O/tests_$n.log 2>&1
  rc=$?; echo "tests [$n]: $(tail -1 $O/tests_$n.log)"; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error" $O/tests_$n.log | head; exit $rc; }
done
SETS=""
for n in $LIBS; do SETS="$SETS MOEVA_MI355X_LIB=$(path $n)"; done
[ -n "$LIBS" ] && { SETS="$SETS" REPS=${REPS:-2} STEPS=${STEPS:-4} bash tools/gpu_ab_env.sh || exit 1; }
if [ -n "$PHASES" ]; then
  export MOEVA_MI355X_LIB=$L/libmoeva_mi355x_clk.so
  ROWS=${ROWS:-20} GENS=100 bash tools/gpu_genc_phases.sh || exit 1
  GENS="50 1000" bash tools/gpu_surv_phases.sh || exit 1
fi
exit 0
