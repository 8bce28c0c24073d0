#!/bin/bash
# k_genc -> k_mlp2 hand-off after the compact layout: fp64 genes (xml_direct, default) vs
# the fp32 ML rows k_genc writes (MV_XML=1), and k_mlp2's gene staging (MV_MLP_CO=0).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
SETS="MV_DEFAULT=1 MV_XML=1 MV_MLP_CO=0" REPS=2 STEPS=5 bash tools/gpu_ab_env.sh
