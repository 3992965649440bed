#!/bin/bash
# Round 3: the commit-row parity cases (comb, latency path, host / device encodings)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_msm.py -k "commit_rows" > gpurun_out/t_zx.log 2>&1
rc=$?; tail -1 gpurun_out/t_zx.log; exit $rc
