#!/bin/bash
# Round-4 fault hunt, step 4 (after the fix): the whole GPU suite with the 4-waves checks
# build (every test also asserts that no device index check failed), then with the plain
# 4-waves build -- the round-3 reproducer.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/fault
L=$PWD/moeva2-ijcai22-replication_amd/lib
PYT="python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests"
MV_ASSERT_CHECKS=1 MOEVA_MI355X_LIB=$L/libmoeva_mi355x_chk4.so timeout -k 10 500 $PYT \
  > gpurun_out/fault/chk4_suite.log 2>&1 || { tail -n 30 gpurun_out/fault/chk4_suite.log; exit 1; }
tail -n 2 gpurun_out/fault/chk4_suite.log
MOEVA_MI355X_LIB=$L/libmoeva_mi355x_w4.so timeout -k 10 500 $PYT \
  > gpurun_out/fault/w4_suite.log 2>&1 || { tail -n 30 gpurun_out/fault/w4_suite.log; exit 1; }
tail -n 2 gpurun_out/fault/w4_suite.log
