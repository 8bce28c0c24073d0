#!/bin/bash
# A/B of a library variant (MOEVA_MI355X_LIB=$VARIANT) against the default build on one box:
# its GPU tests, then default / variant bench lines (4 groups) alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/libab; mkdir -p $O
V=${VARIANT:?}
MOEVA_MI355X_LIB=$V timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 2 > $O/def.json 2> $O/def.log || exit 1
  echo "default $(python3 tools/show_bench.py $O/def.json | head -1)"
  MOEVA_MI355X_LIB=$V timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 2 > $O/var.json 2> $O/var.log || exit 1
  echo "variant $(python3 tools/show_bench.py $O/var.json | head -1)"
done
