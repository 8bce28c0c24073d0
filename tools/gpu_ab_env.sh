#!/bin/bash
# A/B of engine environment switches on the headline (4 state groups, no profiling):
#   SETS="MV_MLP_WAVES=4 MV_MLP_WAVES=8" bash tools/gpu_ab_env.sh   (comma-separated per set)
# Alternates the sets REPS times (default 2) so box drift hits both.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/ab; mkdir -p $O
for r in $(seq 1 ${REPS:-2}); do
  for set in $SETS; do
    envs=$(eval echo "$set" | tr "," " ")
    tag=$(echo $set | sed 's|[^,=]*/||g; s|libmoeva_mi355x_||g; s|\.so||g')
    env $envs timeout -k 10 200 python -u bench.py --steps ${STEPS:-6} --warmup 1 --no-cpu-baseline --no-configs ${BENCH_ARGS:-} > "$O/$tag.$r.json" 2> "$O/$tag.$r.log" || exit 1
    echo "$tag rep $r: $(python3 -c "import json;d=json.load(open('$O/$tag.$r.json'));print(round(d['value']/1e6,2), 'M evals/s', {k: round(v*1000,1) for k,v in d['kernels_avg_ms_per_generation'].items() if not isinstance(v, str)})")"
  done
done
