#!/bin/bash
# k_bullet_comb phases (scripts/micro/bullet_comb_phases.hip): _a = the committed recode, plain = branchless recode
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
{ echo "== a (shift-register recode)"; timeout -k 10 150 ./scripts/micro/bullet_comb_phases_a; } > gpurun_out/bcomb_phases.txt 2>&1 || { cat gpurun_out/bcomb_phases.txt; exit 1; }
{ echo "== b (branchless recode)"; timeout -k 10 150 ./scripts/micro/bullet_comb_phases; } >> gpurun_out/bcomb_phases.txt 2>&1 || { cat gpurun_out/bcomb_phases.txt; exit 1; }
cat gpurun_out/bcomb_phases.txt
