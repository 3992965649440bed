#!/bin/bash
# round-5 profiles of the current tree: kernel stats + PMC traffic of the headline and of each single-GPU extra
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=r05_snark_ PROF=1 PMC=1 bash scripts/gpu_run.sh || exit 1
bash scripts/gpu_profiles.sh || exit 1
ls gpurun_out | grep -i "pmc_traffic\|prof$"
