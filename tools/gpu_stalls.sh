#!/bin/bash
# Stall breakdown of the chain kernels (one state group, 20 generations): where wave time
# goes (active / parked on waitcnt or barrier / issue-stalled) and the instruction mix.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
W="${WORKLOAD:-rq1.botnet.static}"
O=gpurun_out/stalls/$W
mkdir -p $O
BA="--workload $W ${BENCH_ARGS:-} --steps 1 --warmup 0 --no-cpu-baseline --n-gen 20 --groups 1"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --kernel-trace -d $O/p1 -o run --output-format csv -- python3 bench.py $BA > $O/p1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES GRBM_GUI_ACTIVE --kernel-trace -d $O/p2 -o run --output-format csv -- python3 bench.py $BA > $O/p2.log 2>&1 || exit $?
python3 tools/pmc_summary.py $(find $O/p1 $O/p2 -name '*counter_collection.csv') > $O/stalls.txt 2>&1
cat $O/stalls.txt
