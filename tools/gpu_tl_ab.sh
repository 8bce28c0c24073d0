#!/bin/bash
# Kernel-trace timeline (default state groups, 200 generations) per value of an env knob:
#   KNOB=MV_MLPX VALUES="1 0" bash tools/gpu_tl_ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/tlab; mkdir -p $O
for v in ${VALUES}; do
  export $KNOB=$v
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tl$v -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --n-gen 200 > $O/tl$v.log 2>&1 || exit 1
  echo "$KNOB=$v"; python3 tools/timeline.py $(find $O/tl$v -name '*kernel_trace.csv' | head -1) | tee $O/timeline$v.txt
done
