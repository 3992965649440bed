#!/bin/bash
# round-5 GPU call: pool burst cost on the box (pinned), library A/B (pool hot words on their own lines + 64-unit
# slices vs the previous commit), host-path Bullet threshold A/B on the new build
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
(cd scripts/micro && timeout -k 10 120 ./parts_finals_cpu 176 pin > ../../gpurun_out/pf_pin.txt 2>&1) || exit 1
grep -i "pin\|empty\|niels_sum8\|ext_sum8\|entries" gpurun_out/pf_pin.txt
T=300 bash scripts/session_r05.sh tests "test_gpu_snark and not round_forms" || exit 1
timeout -k 10 700 bash scripts/ab_lib.sh lib/libspg_prev.so lib/libspg.so 3 > gpurun_out/ab_lib8.txt 2>&1 || { cat gpurun_out/ab_lib8.txt; exit 1; }
cat gpurun_out/ab_lib8.txt
T=500 bash scripts/session_r05.sh ab SPG_BULLET_HOST_MAX "32 128" 2 > gpurun_out/ab_hostmax2.txt 2>&1 || { tail gpurun_out/ab_hostmax2.txt; exit 1; }
grep "SPG_" gpurun_out/ab_hostmax2.txt
