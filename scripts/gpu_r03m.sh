#!/bin/bash
# Round 3: host cost of HIP calls (launch, copies, events), default and with kernel arguments in device memory
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 60 ./scripts/micro/launch_cost > gpurun_out/launch_cost.txt 2>&1 || exit $?
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 60 ./scripts/micro/launch_cost > gpurun_out/launch_cost_devk.txt 2>&1 || exit $?
HIP_FORCE_DEV_KERNARG=0 timeout -k 10 60 ./scripts/micro/launch_cost > gpurun_out/launch_cost_hostk.txt 2>&1 || exit $?
echo default; tail -10 gpurun_out/launch_cost.txt; echo devk; tail -10 gpurun_out/launch_cost_devk.txt; echo hostk; tail -10 gpurun_out/launch_cost_hostk.txt
