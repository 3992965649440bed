#!/bin/bash
# branchless comb recode in k_bullet_comb / k_comb_msm_parts: parity (SNARK goldens, Bullet paths, MSM comb parts),
# then the headline ABBA against the committed build (lib/libspg_head.so)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_snark.py tests/test_gpu_msm.py \
  -k "golden or bullet or comb or parts or dot" > gpurun_out/t51.log 2>&1
rc=$?; tail -3 gpurun_out/t51.log; [ $rc = 0 ] || exit $rc
bash scripts/ab_lib2.sh lib/libspg_head.so lib/libspg.so 3 > gpurun_out/ab51.txt && cat gpurun_out/ab51.txt
