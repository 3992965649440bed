#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
T=900 bash scripts/session_r05.sh tests "thread_form or test_round_forms or test_snark_2e20_headline or test_config4 or test_bullet_paths" || exit 1
BENCH_ARGS="--workload r1cs --config r1cs_2e22_p8" timeout -k 10 500 bash scripts/ab_env2.sh SPG_P1_ROWS 0 1 3 > gpurun_out/ab15_rows.txt 2>&1 || { cat gpurun_out/ab15_rows.txt; exit 1; }
cat gpurun_out/ab15_rows.txt
