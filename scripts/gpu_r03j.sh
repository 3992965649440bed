#!/bin/bash
# Round 3: phase probes of the lane-form large-MSM accumulation
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
SPG_BIG_PROBE=1 timeout -k 10 200 python bench.py --workload msm --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/msm_probe.json 2> gpurun_out/msm_probe.err
rc=$?; grep "big accum\|blockIdx" gpurun_out/msm_probe.err | tail -9; exit $rc
