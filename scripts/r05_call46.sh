#!/bin/bash
# layer launch plan knobs: step costs 18,25,30 vs 18,22,26; triple_max 384 vs 192 (ABBA, 3 blocks each)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
bash scripts/ab_env2.sh SPG_STEP_COSTS 18,25,30 18,22,26 3 > gpurun_out/ab46a.txt && cat gpurun_out/ab46a.txt &&
bash scripts/ab_env2.sh SPG_TRIPLE_MAX 384 192 3 > gpurun_out/ab46b.txt && cat gpurun_out/ab46b.txt
