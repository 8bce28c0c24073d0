#!/bin/bash
# Round-4 fault hunt, step 3: the default library's GPU suite, then the 4-waves checks build
# (final-offset checks at every k_genc global access) on the failing case, serialised.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/fault
L=$PWD/moeva2-ijcai22-replication_amd/lib
PYT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
if [ -z "$SKIP_SUITE" ]; then
timeout -k 10 400 $PYT -m gpu tests > gpurun_out/fault/suite.log 2>&1 || { tail -n 30 gpurun_out/fault/suite.log; exit 1; }
tail -n 2 gpurun_out/fault/suite.log
fi
T="tests/test_gpu_parity.py::test_attack_chain_deterministic[botnet_augmented-3-43-20-5-2-two_point]"
MOEVA_MI355X_LIB=$L/libmoeva_mi355x_${V:-chk4}.so AMD_SERIALIZE_KERNEL=3 \
  timeout -k 10 200 $PYT "$T" > gpurun_out/fault/${V:-chk4}_aug3.log 2>&1
rc=$?
grep -n "Error\|error\|check" gpurun_out/fault/${V:-chk4}_aug3.log | tail -n 12
exit $rc
