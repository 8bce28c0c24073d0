#!/bin/bash
# A/B: whole-attack kernel at 256 vs 512 threads per workgroup, and the chain.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/att
timeout -k 10 300 python -u tools/attack_ab.py --n-gen 200 --reps 2 --modes whole,chain > gpurun_out/att/t256.log 2>&1 || { tail gpurun_out/att/t256.log; exit 1; }
grep '^{' gpurun_out/att/t256.log
MOEVA_MI355X_LIB=$PWD/moeva2-ijcai22-replication_amd/lib/libmoeva_mi355x_att512.so timeout -k 10 300 python -u tools/attack_ab.py --n-gen 200 --reps 2 --modes whole,chain > gpurun_out/att/t512.log 2>&1 || { tail gpurun_out/att/t512.log; exit 1; }
grep '^{' gpurun_out/att/t512.log
