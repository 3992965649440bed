#!/bin/bash
# round-5 GPU call: the whole GPU suite on the current build, then library A/Bs against the IFMA commit's build
# (SNARK headline, config 4)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
T=900 TAG=full_ bash scripts/session_r05.sh tests "gpu" || exit 1
timeout -k 10 600 bash scripts/ab_lib.sh lib/libspg_prev.so lib/libspg.so 3 > gpurun_out/ab_lib12.txt 2>&1 || { cat gpurun_out/ab_lib12.txt; exit 1; }
cat gpurun_out/ab_lib12.txt
BENCH_ARGS="--workload r1cs --config r1cs_2e22_p8" timeout -k 10 600 bash scripts/ab_lib.sh lib/libspg_prev.so lib/libspg.so 3 \
  > gpurun_out/ab_lib12_r1cs.txt 2>&1 || { cat gpurun_out/ab_lib12_r1cs.txt; exit 1; }
cat gpurun_out/ab_lib12_r1cs.txt
