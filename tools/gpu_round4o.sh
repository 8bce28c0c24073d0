#!/bin/bash
# Mating-major offspring chunks: GPU suite, headline + SBX A/B against the strided variant,
# then a PMC FETCH/WRITE pass of the new k_genc.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r4 gpurun_out/ab
timeout -k 10 800 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r4/suite_pairs.log 2>&1
rc=$?; tail -n 3 gpurun_out/r4/suite_pairs.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/r4/suite_pairs.log | head -30; exit $rc; }
L=$PWD/moeva2-ijcai22-replication_amd/lib
SETS="MV_PAIRS=1 MOEVA_MI355X_LIB=$L/libmoeva_mi355x_strided.so" REPS=2 STEPS=6 bash tools/gpu_ab_env.sh || exit 1
SETS="MV_PAIRS=1 MOEVA_MI355X_LIB=$L/libmoeva_mi355x_strided.so" REPS=1 STEPS=3 BENCH_ARGS="--crossover sbx" bash tools/gpu_ab_env.sh || exit 1
O=gpurun_out/pairs; mkdir -p $O
BA="--workload rq1.botnet.static --steps 1 --warmup 0 --no-cpu-baseline --n-gen 20 --groups 1"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc_fetch -o run --output-format csv -- python3 bench.py $BA > $O/pmc_fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmc_write -o run --output-format csv -- python3 bench.py $BA > $O/pmc_write.log 2>&1 || exit $?
python3 tools/pmc_traffic.py $O/pmc_traffic_pairs.json $(find $O/pmc_fetch $O/pmc_write -name '*counter_collection.csv') > $O/pmc_traffic.log 2>&1
head -8 $O/pmc_traffic.log
