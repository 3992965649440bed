#!/bin/bash
# Bullet comb fold: both operands loaded, then selected (no dependent pointer load): phases (a = recode only,
# plain = + operand loads), parity, headline ABBA against the build before the recode (lib/libspg_head.so)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
{ echo "== a (branchless recode)"; timeout -k 10 150 ./scripts/micro/bullet_comb_phases_a; } > gpurun_out/bcomb_phases2.txt 2>&1 || { cat gpurun_out/bcomb_phases2.txt; exit 1; }
{ echo "== b (+ both fold operands loaded, then selected)"; timeout -k 10 150 ./scripts/micro/bullet_comb_phases; } >> gpurun_out/bcomb_phases2.txt 2>&1 || { cat gpurun_out/bcomb_phases2.txt; exit 1; }
grep "gap   0" gpurun_out/bcomb_phases2.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_snark.py tests/test_gpu_msm.py \
  -k "golden or bullet or comb or parts or dot" > gpurun_out/t54.log 2>&1
rc=$?; tail -2 gpurun_out/t54.log; [ $rc = 0 ] || exit $rc
bash scripts/ab_lib2.sh lib/libspg_head.so lib/libspg.so 3 > gpurun_out/ab54.txt && cat gpurun_out/ab54.txt
