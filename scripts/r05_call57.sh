#!/bin/bash
# field products with the carry additions trailing by two (field.hpp MacAcc: 1,084 -> 681 s_nop in k_bullet_comb):
# Bullet phases (a = before), the full -m gpu suite (every kernel's arithmetic), headline ABBA (lib/libspg_head.so = before)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
{ echo "== a (mac_ov)"; timeout -k 10 150 ./scripts/micro/bullet_comb_phases_a; } > gpurun_out/bcomb_phases3.txt 2>&1 || { cat gpurun_out/bcomb_phases3.txt; exit 1; }
{ echo "== b (MacAcc)"; timeout -k 10 150 ./scripts/micro/bullet_comb_phases; } >> gpurun_out/bcomb_phases3.txt 2>&1 || { cat gpurun_out/bcomb_phases3.txt; exit 1; }
grep "gap   0" gpurun_out/bcomb_phases3.txt
TAG=r05x_ TESTS=1 T_TESTS=900 bash scripts/gpu_run.sh || exit 1
bash scripts/ab_lib2.sh lib/libspg_head.so lib/libspg.so 3 > gpurun_out/ab57.txt && cat gpurun_out/ab57.txt
