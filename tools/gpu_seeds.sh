#!/bin/bash
# Per-state device success over seeds (tools/seed_states.py), then a short bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for spec in ${SEED_SPECS:-g1000:32:1000}; do
  IFS=: read tag n g <<< "$spec"
  timeout -k 10 300 python -u tools/seed_states.py ${FIXTURE:-e2e_botnet_rq1_seeds.npz} $tag $n $g \
    >> gpurun_out/seeds.log 2>&1 || { echo "seed sweep $tag failed rc=$?"; tail -5 gpurun_out/seeds.log; exit 1; }
done
grep -v amdgpu.ids gpurun_out/seeds.log | tail -5
if [ -n "$BENCH" ]; then
  timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --n-gen 200 \
    > gpurun_out/bench.json 2> gpurun_out/bench.log || exit 1
  python3 tools/show_bench.py gpurun_out/bench.json
fi
