#!/bin/bash
# Round-6 iteration on one GPU box: the whole parity suite on the product build, the headline
# A/B of LIBS (tools/gpu_ab_env.sh), the small-attack workloads (WORKLOADS) per library, and
# the survival phase clocks of the clocks builds PHASE_LIBS.  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06; mkdir -p $O
L=moeva2-ijcai22-replication_amd/lib
path() { [ -z "$1" -o "$1" = main ] && echo $L/libmoeva_mi355x.so || echo $L/libmoeva_mi355x_$1.so; }
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $O/gpu_tests.log 2>&1
  rc=$?; echo "tests: $(tail -1 $O/gpu_tests.log)"; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error" $O/gpu_tests.log | head; exit $rc; }
fi
SETS=""
for n in $LIBS; do SETS="$SETS MOEVA_MI355X_LIB=$(path $n)"; done
[ -n "$LIBS" ] && { SETS="$SETS" REPS=${REPS:-2} STEPS=${STEPS:-4} bash tools/gpu_ab_env.sh || exit 1; }
for w in $WORKLOADS; do
  for n in $LIBS; do
    MOEVA_MI355X_LIB=$(path $n) timeout -k 10 300 python -u bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline --no-configs --no-generate > $O/$w.$n.json 2> $O/$w.$n.log || exit 1
    echo "$w [$n]: $(python3 -c "import json;d=json.load(open('$O/$w.$n.json'));print(round(d['value']/1e6,2), 'M evals/s', {k: round(v*1000,1) for k,v in d['kernels_avg_ms_per_generation'].items() if not isinstance(v, str)})")"
  done
done
for n in $PHASE_LIBS; do  # clocks builds (MV_CLOCKS=1), e.g. PHASE_LIBS="clk"
  echo "phases [$n]"
  MOEVA_MI355X_LIB=$(path $n) GENS="${GENS:-1000}" bash tools/gpu_surv_phases.sh || exit 1
done
exit 0
