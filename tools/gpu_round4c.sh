#!/bin/bash
# Clone-heavy survival replay (default library) + survival phase clocks (MV_CLOCKS build).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r4
timeout -k 10 200 python -u -m pytest -v --timeout 120 --timeout-method thread \
  "tests/test_gpu_parity.py::test_survival_bit_exact_on_clone_heavy_botnet_states" \
  "tests/test_gpu_parity.py::test_survival_bit_exact_vs_oracle" > gpurun_out/r4/clones.log 2>&1
grep -E "PASS|FAIL|Error|assert|Mismatch|mismatch|Max abs|x: |y: " gpurun_out/r4/clones.log | head -40
for g in 50 1000; do
  MOEVA_MI355X_LIB=$PWD/moeva2-ijcai22-replication_amd/lib/libmoeva_mi355x_clk.so MV_SURV_PHASES=1 \
    timeout -k 10 200 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --n-gen $g --groups 1 \
    > gpurun_out/r4/sph$g.json 2> gpurun_out/r4/sph$g.log || exit 1
  echo "n_gen=$g"; grep "\[mv\]" gpurun_out/r4/sph$g.log
done
