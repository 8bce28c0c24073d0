#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/fault
MOEVA_MI355X_LIB=$PWD/moeva2-ijcai22-replication_amd/lib/libmoeva_mi355x_chk4.so \
  DUMP_SEEDS=1000,1001,1002 timeout -k 10 300 python -u tools/surv_dump.py > gpurun_out/fault/surv_dump.log 2>&1
rc=$?
tail -n 20 gpurun_out/fault/surv_dump.log
exit $rc
