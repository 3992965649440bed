#!/bin/bash
# round-5 final tree (Bullet recode + fold loads): full -m gpu suite, smoke, the driver's default bench line
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=r05y_ TESTS=1 T_TESTS=900 SMOKE=1 BENCH=1 T_BENCH=600 bash scripts/gpu_run.sh
