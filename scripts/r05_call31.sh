#!/bin/bash
# Bullet parts per workgroup again, with the 8-lane host sums: R 4 vs 8, 4 vs 16 (ABBA, 3 blocks each)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
bash scripts/ab_env2.sh SPG_BCOMB_R 4 8 3 > gpurun_out/ab31a.txt && cat gpurun_out/ab31a.txt &&
bash scripts/ab_env2.sh SPG_BCOMB_R 4 16 3 > gpurun_out/ab31b.txt && cat gpurun_out/ab31b.txt
