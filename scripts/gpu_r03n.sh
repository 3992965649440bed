#!/bin/bash
# Round 3: SNARK bench with kernel arguments in device memory (HIP default here) vs host memory
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
bash scripts/ab_env.sh HIP_FORCE_DEV_KERNARG "1 0" 3
