#!/bin/bash
# A/B of engine environment switches on the headline (4 state groups, no profiling):
#   SETS="MV_MLP_WAVES=4 MV_MLP_WAVES=8" bash tools/gpu_ab_env.sh   (comma-separated per set)
# Alternates the sets REPS times (default 2) so box drift hits both.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/ab; mkdir -p $O
for r in $(seq 1 ${REPS:-2}); do
  for set in $SETS; do
    envs=$(echo $set | tr ',' ' ')
    env $envs timeout -k 10 200 python -u bench.py --steps ${STEPS:-6} --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > $O/$set.$r.json 2> $O/$set.$r.log || exit 1
    echo "$set rep $r: $(python3 -c "import json;d=json.load(open('$O/$set.$r.json'));print(round(d['value']/1e6,2), 'M evals/s')")"
  done
done
