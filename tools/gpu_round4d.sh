#!/bin/bash
# Round 4: GPU suite (default library), checks-build attack over 3 seeds (no device check may
# fail), survival phase clocks (MV_CLOCKS build), headline bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r4
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests \
  -k "not test_success_rate_within_1pp_state_streams or lcld" > gpurun_out/r4/suite.log 2>&1
rc=$?
tail -n 3 gpurun_out/r4/suite.log
[ $rc -ne 0 ] && { grep -E "FAIL|Error" gpurun_out/r4/suite.log | head; exit $rc; }
bash tools/gpu_surv_dump.sh || exit $?
MOEVA_MI355X_LIB=$PWD/moeva2-ijcai22-replication_amd/lib/libmoeva_mi355x_clk.so MV_SURV_PHASES=1 \
  timeout -k 10 200 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --n-gen 50 --groups 1 \
  > gpurun_out/r4/sph50.json 2> gpurun_out/r4/sph50.log || exit 1
grep "\[mv\]" gpurun_out/r4/sph50.log
MOEVA_MI355X_LIB=$PWD/moeva2-ijcai22-replication_amd/lib/libmoeva_mi355x_clknp.so MV_SURV_PHASES=1 \
  timeout -k 10 200 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --n-gen 50 --groups 1 \
  > gpurun_out/r4/sph50np.json 2> gpurun_out/r4/sph50np.log || exit 1
echo "six-compare dominance:"; grep "\[mv\]" gpurun_out/r4/sph50np.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r4/bench.json 2> gpurun_out/r4/bench.log || exit $?
python3 -c "import json;d=json.load(open('gpurun_out/r4/bench.json'));print(d['value'], d['kernels_avg_ms_per_generation'])"
