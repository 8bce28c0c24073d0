#!/bin/bash
# A/B of an engine environment switch (ENVS="NAME=VAL ..." each run against the default):
# per-kernel split with one state group, then the default-groups bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/envab
BA="--steps 1 --warmup 1 --no-cpu-baseline --n-gen ${NGEN:-200} ${BENCH_ARGS:-}"
for e in default ${ENVS}; do
  for g in 1 0; do
    GA=""; [ $g = 1 ] && GA="--groups 1"
    if [ $e = default ]; then
      timeout -k 10 200 python -u bench.py $BA $GA > gpurun_out/envab/r.json 2> gpurun_out/envab/r.log || exit $?
    else
      env $e timeout -k 10 200 python -u bench.py $BA $GA > gpurun_out/envab/r.json 2> gpurun_out/envab/r.log || exit $?
    fi
    echo "$e groups=$g $(python3 tools/show_bench.py gpurun_out/envab/r.json | head -1)"
  done
done
