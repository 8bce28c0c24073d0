#!/bin/bash
# PMC passes over a short single-group bench run (one counter group per rocprofv3 run,
# kernel-trace only, no sys/runtime traces), then per-kernel means (tools/pmc_summary.py).
#   PMC_GROUPS="<counters>\n<counters>..." PMC_ARGS="<bench.py args>" bash tools/gpu_pmc.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${PMC_OUT:-pmc}; mkdir -p $O
ARGS="${PMC_ARGS:---steps 1 --warmup 0 --no-cpu-baseline --n-gen 20 --groups 1}"
i=0
while read -r group; do
  [ -z "$group" ] && continue
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $group --kernel-trace -d $O/p$i -o run \
     --output-format csv -- python3 bench.py $ARGS > $O/p$i.log 2>&1
  rc=$?; echo "pass $i ($group) rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done <<< "${PMC_GROUPS:-SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD
FETCH_SIZE
WRITE_SIZE
SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE}"
python3 tools/pmc_summary.py $O/p*/run_counter_collection.csv | grep -E "k_gen|k_cons|k_mlp|k_survive|k_narrow"
