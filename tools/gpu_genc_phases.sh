#!/bin/bash
# k_genc phase split (MV_GEN_PHASES=1: clock64 per workgroup of the last generation, one
# state group), for each MV_VARY_ROWS in ROWS.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/gph; mkdir -p $O
for r in ${ROWS:-32}; do
  MV_VARY_ROWS=$r MV_GEN_PHASES=1 timeout -k 10 200 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --n-gen ${GENS:-100} --groups 1 > $O/r$r.json 2> $O/r$r.log || exit 1
  echo "rows cap $r"; grep "\[mv\] k_genc" $O/r$r.log
done
