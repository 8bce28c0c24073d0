#!/bin/bash
# Development sweep: state groups x rows per k_gen/k_cons workgroup, + survival phase split.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/sweep; mkdir -p $O
for G in ${GS:-2 4 6 8}; do for R in ${RS:-16 32 64}; do
  MV_GROUPS=$G MV_VARY_ROWS=$R timeout -k 10 120 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/g${G}_r${R}.json 2> $O/g${G}_r${R}.log
  rc=$?; case $rc in 0) ;; *) echo "G=$G R=$R rc=$rc"; exit $rc;; esac
  echo "G=$G R=$R $(python3 tools/show_bench.py $O/g${G}_r${R}.json | head -1)"
done; done
for R in ${RS:-16 32 64}; do
  MV_VARY_ROWS=$R timeout -k 10 120 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --groups 1 > $O/g1_r${R}.json 2> $O/g1_r${R}.log || exit 1
  echo "G=1 R=$R $(python3 tools/show_bench.py $O/g1_r${R}.json | head -1)"
done
MV_SURV_PHASES=1 timeout -k 10 120 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --n-gen 50 > $O/phases.json 2> $O/phases.log || exit 1
grep "\[mv\]" $O/phases.log
