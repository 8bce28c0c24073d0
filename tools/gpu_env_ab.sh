#!/bin/bash
# Headline bench (default 4 state groups) per value of an engine env knob:
#   KNOB=MV_VARY_ROWS VALUES="32 16 12 10" bash tools/gpu_env_ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/envab; mkdir -p $O
for v in ${VALUES}; do
  env $KNOB=$v timeout -k 10 200 python -u bench.py --steps ${STEPS:-2} --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > $O/$KNOB.$v.json 2> $O/$KNOB.$v.log || exit 1
  echo "$KNOB=$v $(python3 -c "import json;d=json.load(open('$O/$KNOB.$v.json'));print(round(d['value']/1e6,1),'M evals/s', {k:round(v*1000,1) for k,v in d['kernels_avg_ms_per_generation'].items() if k!='dominant'})")"
done
