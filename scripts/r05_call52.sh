#!/bin/bash
# tiny Bullet rounds without the LDS tree (SPG_BCOMB_NOTREE): parity under the switch, then headline ABBA 0 vs 4
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
SPG_BCOMB_NOTREE=4 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_snark.py \
  -k "golden or bullet" > gpurun_out/t52.log 2>&1
rc=$?; tail -3 gpurun_out/t52.log; [ $rc = 0 ] || exit $rc
bash scripts/ab_env2.sh SPG_BCOMB_NOTREE 0 4 3 > gpurun_out/ab52.txt && cat gpurun_out/ab52.txt
