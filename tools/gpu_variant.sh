#!/bin/bash
# Per-kernel split (one state group, 200 generations) of the default library and of a
# development variant library (VARIANT=<suffix>: lib/libmoeva_mi355x_<suffix>.so).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/var
BA="--steps 1 --warmup 1 --no-cpu-baseline --n-gen 200 --groups 1 ${BENCH_ARGS:-}"
timeout -k 10 200 python -u bench.py $BA > gpurun_out/var/base.json 2> gpurun_out/var/base.log || exit $?
echo "base    $(python3 tools/show_bench.py gpurun_out/var/base.json | head -1)"
for v in ${VARIANT}; do
MOEVA_MI355X_LIB=$PWD/moeva2-ijcai22-replication_amd/lib/libmoeva_mi355x_$v.so timeout -k 10 200 python -u bench.py $BA > gpurun_out/var/$v.json 2> gpurun_out/var/$v.log || exit $?
echo "$v $(python3 tools/show_bench.py gpurun_out/var/$v.json | head -1)"
done
