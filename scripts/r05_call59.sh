#!/bin/bash
# round-5 final tree (MacAcc field products merged; library identical to the one r05_call58 tested: 204 passed):
# smoke and the driver's default bench line
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=r05w_ SMOKE=1 BENCH=1 T_BENCH=600 bash scripts/gpu_run.sh
