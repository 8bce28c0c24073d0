#!/bin/bash
# Kernel-trace timelines (default state groups, 200 generations) for a list of env settings:
#   SETS="MV_MLPX=1,MV_MLPX_NR=2 MV_MLPX=0" bash tools/gpu_tl_env.sh   (comma-separated per set)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/tlenv; mkdir -p $O
i=0
for set in ${SETS}; do
  i=$((i+1))
  ( for kv in ${set//,/ }; do export "$kv"; done
    timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tl$i -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --n-gen 200 > $O/tl$i.log 2>&1 ) || exit 1
  echo "== $set"; python3 tools/timeline.py $(find $O/tl$i -name '*kernel_trace.csv' | head -1) | tee $O/timeline$i.txt
done
