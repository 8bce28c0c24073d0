#!/bin/bash
# The remaining config lines of gpu_configs.sh (bf16, k_mlpw, scale-out, wide) -> gpurun_out/configs/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/configs; mkdir -p $O
run() {  # name, timeout, args...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t python -u bench.py "$@" > $O/$n.json 2> $O/$n.log
  local rc=$?; echo "$n rc=$rc $(python3 tools/show_bench.py $O/$n.json 2>/dev/null | head -1)"
  case $rc in 0) ;; *) exit $rc;; esac
}
run c2_botnet_bf16 300 --workload rq1.botnet.static --mlp-dtype bf16 --steps 2 --warmup 1 --no-cpu-baseline
run c4_lcld_scaleout 600 --workload synthetic.lcld.scaleout --steps 1 --warmup 1 --no-cpu-baseline
run c5_botnet_wide_bf16 600 --workload synthetic.botnet.wide --mlp-dtype bf16 --steps 1 --warmup 1 --no-cpu-baseline
run c5_botnet_wide_fp32 600 --workload synthetic.botnet.wide --steps 1 --warmup 1 --no-cpu-baseline
