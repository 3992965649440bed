#!/bin/bash
# Round 3: per-exchange latency of the SPMD transports
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 300 python scripts/comm_latency.py > gpurun_out/comm_latency.json 2> gpurun_out/comm_latency.err
rc=$?; cat gpurun_out/comm_latency.json; tail -3 gpurun_out/comm_latency.err; exit $rc
