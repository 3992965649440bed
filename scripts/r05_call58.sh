#!/bin/bash
# experiment (branch field-carry-pipeline): field products with the carry additions trailing by two, built as
# lib/libspg_macacc.so: Bullet phases (a = main), the full -m gpu suite on that library, headline ABBA against main
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
{ echo "== a (main: mac_ov)"; timeout -k 10 150 ./scripts/micro/bullet_comb_phases_a; } > gpurun_out/bcomb_phases3.txt 2>&1 || { cat gpurun_out/bcomb_phases3.txt; exit 1; }
{ echo "== b (MacAcc)"; timeout -k 10 150 ./scripts/micro/bullet_comb_phases; } >> gpurun_out/bcomb_phases3.txt 2>&1 || { cat gpurun_out/bcomb_phases3.txt; exit 1; }
grep "gap   0" gpurun_out/bcomb_phases3.txt
SPG_LIB=$R/spartan-parallel_amd/lib/libspg_macacc.so TAG=r05x_ TESTS=1 T_TESTS=900 bash scripts/gpu_run.sh || exit 1
bash scripts/ab_lib2.sh lib/libspg.so lib/libspg_macacc.so 3 > gpurun_out/ab58.txt && cat gpurun_out/ab58.txt
