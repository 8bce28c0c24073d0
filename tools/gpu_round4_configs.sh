#!/bin/bash
# Round 4: one bench line per BASELINE config (tools/gpu_configs.sh), then a rocprofv3
# kernel-stats pass and FETCH_SIZE / WRITE_SIZE PMC passes of configs[3] (the survival-bound
# scale-out), one state group, 5 generations.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_configs.sh || exit $?
O=gpurun_out/c4prof; mkdir -p $O
BA="--workload synthetic.lcld.scaleout --steps 1 --warmup 0 --no-cpu-baseline --n-gen 5 --groups 1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py $BA > $O/prof.log 2>&1 || exit $?
cp $(find $O/prof -name '*kernel_stats.csv' | head -1) $O/kernel_stats.csv; head -6 $O/kernel_stats.csv
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc_fetch -o run --output-format csv -- python3 bench.py $BA > $O/pmc_fetch.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmc_write -o run --output-format csv -- python3 bench.py $BA > $O/pmc_write.log 2>&1 || exit $?
python3 tools/pmc_traffic.py $O/pmc_traffic_synthetic.lcld.scaleout_chain.json $(find $O/pmc_fetch $O/pmc_write -name '*counter_collection.csv') > $O/pmc_traffic.log 2>&1
cat $O/pmc_traffic.log
