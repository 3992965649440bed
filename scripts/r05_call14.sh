#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
T=300 bash scripts/session_r05.sh tests "test_gpu_r1cs" || exit 1
BENCH_ARGS="--workload r1cs --config r1cs_2e22_p8" timeout -k 10 500 bash scripts/ab_env2.sh SPG_SC_GRID 1024 2048 2 > gpurun_out/ab14_grid.txt 2>&1 || { cat gpurun_out/ab14_grid.txt; exit 1; }
cat gpurun_out/ab14_grid.txt
BENCH_ARGS="--workload r1cs --config r1cs_2e22_p8" timeout -k 10 500 bash scripts/ab_env2.sh SPG_SC_GRID 1024 1536 2 > gpurun_out/ab14_grid2.txt 2>&1 || { cat gpurun_out/ab14_grid2.txt; exit 1; }
cat gpurun_out/ab14_grid2.txt
timeout -k 10 700 bash scripts/ab_env2.sh SPG_BCOMB_R 2 4 2 > gpurun_out/ab14_r.txt 2>&1 || { cat gpurun_out/ab14_r.txt; exit 1; }
cat gpurun_out/ab14_r.txt
