#!/bin/bash
# Round 4 v2 (compact layout): one bench line per BASELINE config (tools/gpu_configs.sh) and
# the wide fp32 line, then configs[3]'s rocprofv3 kernel stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
rm -rf gpurun_out/configs
bash tools/gpu_configs.sh || exit $?
O=gpurun_out/configs
timeout -k 10 600 python -u bench.py --workload synthetic.botnet.wide --steps 1 --warmup 1 --no-cpu-baseline > $O/c5_botnet_wide_fp32.json 2> $O/c5_botnet_wide_fp32.log || exit $?
python3 tools/show_bench.py $O/c5_botnet_wide_fp32.json | head -1
