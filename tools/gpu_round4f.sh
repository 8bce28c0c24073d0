#!/bin/bash
# LDS-footprint sensitivity of the headline: each kernel's dynamic LDS request padded by
# 16 KiB (MV_LDS_PAD_*), against no padding.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
SETS="MV_LDS_PAD_GENC=0 MV_LDS_PAD_GENC=16384 MV_LDS_PAD_MLP=16384 MV_LDS_PAD_SURV=16384" REPS=1 STEPS=6 bash tools/gpu_ab_env.sh
for f in gpurun_out/ab/MV_LDS_PAD*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f', {k: round(v*1000,1) for k,v in d['kernels_avg_ms_per_generation'].items() if k!='dominant'})"; done
