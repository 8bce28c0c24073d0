#!/bin/bash
# One bench line per BASELINE.json config (configs[0..4]) on one GPU -> gpurun_out/configs/,
# plus the bf16 perf-mode lines (labelled in their JSON).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/configs; mkdir -p $O
run() {  # name, timeout, args...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t python -u bench.py "$@" > $O/$n.json 2> $O/$n.log
  local rc=$?; echo "$n rc=$rc $(python3 tools/show_bench.py $O/$n.json 2>/dev/null | head -1)"
  case $rc in 0) ;; *) exit $rc;; esac
}
run c1_lcld_static_g100 200 --workload rq1.lcld.static --steps 3 --warmup 1 --cpu-gens 100
run c1_lcld_static_g1000 300 --workload rq1.lcld.static --n-gen 1000 --steps 2 --warmup 1 --no-cpu-baseline
run c3_lcld_augmented 300 --workload rq4.lcld.moeva_augmented --steps 2 --warmup 1 --cpu-gens 100
run c2_botnet_bf16 300 --workload rq1.botnet.static --mlp-dtype bf16 --steps 2 --warmup 1 --no-cpu-baseline
MV_MLPW=1 run c2_botnet_bf16_mlpw 300 --workload rq1.botnet.static --mlp-dtype bf16 --steps 2 --warmup 1 --no-cpu-baseline
run c4_lcld_scaleout 600 --workload synthetic.lcld.scaleout --steps 1 --warmup 1 --no-cpu-baseline
run c2_botnet_sbx 300 --workload rq1.botnet.static --crossover sbx --steps 2 --warmup 1 --no-cpu-baseline
run c5_botnet_wide_bf16 600 --workload synthetic.botnet.wide --mlp-dtype bf16 --steps 1 --warmup 1 --no-cpu-baseline
