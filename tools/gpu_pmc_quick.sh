#!/bin/bash
# One PMC pass per counter group over a short bench run; prints per-kernel means.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmcq
ARGS="${PMC_ARGS:---steps 1 --warmup 0 --no-cpu-baseline --n-gen 20}"
i=0
while read -r group; do
  [ -z "$group" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $group --kernel-trace -d gpurun_out/pmcq/p$i -o run \
     --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmcq/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  case $rc in 124|134|137|139) echo stop; exit $rc;; esac
done <<< "${PMC_GROUPS:-SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD
FETCH_SIZE
WRITE_SIZE
SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE}"
python3 tools/pmc_summary.py gpurun_out/pmcq/p*/run_counter_collection.csv | grep -E "k_gen|k_cons|k_mlp|k_survive"
