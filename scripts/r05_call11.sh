#!/bin/bash
# round-5 GPU call: parity of the fused product-tree tops (round forms, SPARK tests), A/B of SPG_TREE_TOP
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
T=600 bash scripts/session_r05.sh tests "test_round_forms or test_gpu_spark" || exit 1
T=500 bash scripts/session_r05.sh ab SPG_TREE_TOP "0 1024" 3 > gpurun_out/ab_tree.txt 2>&1 || { tail gpurun_out/ab_tree.txt; exit 1; }
grep "SPG_" gpurun_out/ab_tree.txt
