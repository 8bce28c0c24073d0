#!/bin/bash
# Schedule knobs after the compact layout: state groups (MV_GROUPS) and offspring rows per
# k_genc workgroup (MV_VARY_ROWS), one rep each, then the default again.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
SETS="MV_DEFAULT=1 MV_GROUPS=3 MV_VARY_ROWS=25 MV_VARY_ROWS=17 MV_VARY_ROWS=34 MV_DEFAULT=2" REPS=1 STEPS=5 bash tools/gpu_ab_env.sh
