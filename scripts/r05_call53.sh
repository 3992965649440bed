#!/bin/bash
# final-tree profiles: kernel stats + PMC traffic of the headline (Bullet recode) and the row batch (13-bit comb)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=r05h_snark_ PROF=1 PMC=1 bash scripts/gpu_run.sh || exit 1
PROFILE_WORKLOADS="rows:--workload rows" bash scripts/gpu_profiles.sh || exit 1
ls gpurun_out | grep -i "pmc_traffic"
