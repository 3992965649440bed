#!/bin/bash
# Round 3: host breakdown after the host-path changes, and the host/device Bullet threshold A/B
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
SPG_TRACE=2 timeout -k 10 200 python scripts/trace_snark.py > gpurun_out/trace2.out 2> gpurun_out/trace2.err || exit $?
SPG_TRACE=1 timeout -k 10 200 python scripts/trace_snark.py > gpurun_out/trace1.out 2> gpurun_out/trace1.err || exit $?
tail -1 gpurun_out/trace1.err
bash scripts/ab_env.sh SPG_BULLET_HOST_MAX "32 16 64" 3
