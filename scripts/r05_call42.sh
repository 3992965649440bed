#!/bin/bash
# round-5 final profiles: kernel stats + PMC traffic of the headline, config 2 (msm, rows)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=r05g_snark_ PROF=1 PMC=1 bash scripts/gpu_run.sh || exit 1
PROFILE_WORKLOADS="msm:--workload msm|rows:--workload rows" bash scripts/gpu_profiles.sh || exit 1
ls gpurun_out | grep -i "pmc_traffic"
