#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
BENCH_ARGS="--workload r1cs --config r1cs_2e22_p8" timeout -k 10 700 bash scripts/ab_lib2.sh lib/libspg_prev.so lib/libspg.so 3 \
  > gpurun_out/ab13_r1cs.txt 2>&1 || { cat gpurun_out/ab13_r1cs.txt; exit 1; }
cat gpurun_out/ab13_r1cs.txt
timeout -k 10 900 bash scripts/ab_lib2.sh lib/libspg_prev.so lib/libspg.so 2 > gpurun_out/ab13_snark.txt 2>&1 || { cat gpurun_out/ab13_snark.txt; exit 1; }
cat gpurun_out/ab13_snark.txt
