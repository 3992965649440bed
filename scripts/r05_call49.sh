#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
uptime
bash scripts/ab_env2.sh SPG_COMB_C 12 13 4 > gpurun_out/ab49.txt && cat gpurun_out/ab49.txt
