#!/bin/bash
# round-5 GPU call: with the IFMA host sums, A/B of the host slice size and of the host-path Bullet threshold
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
T=500 bash scripts/session_r05.sh ab SPG_SLICE_MIN "8 32 64" 2 > gpurun_out/ab_slice.txt 2>&1 || { tail gpurun_out/ab_slice.txt; exit 1; }
grep "SPG_" gpurun_out/ab_slice.txt
T=500 bash scripts/session_r05.sh ab SPG_BULLET_HOST_MAX "32 64 128" 2 > gpurun_out/ab_hostmax.txt 2>&1 || { tail gpurun_out/ab_hostmax.txt; exit 1; }
grep "SPG_" gpurun_out/ab_hostmax.txt
