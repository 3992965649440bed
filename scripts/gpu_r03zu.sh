#!/bin/bash
# Round 3: the driver's smoke() and the drop-in / dist GPU tests on the final tree
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dropin.py tests/test_gpu_dist.py tests/test_gpu_verify.py > gpurun_out/t_zu.log 2>&1
rc=$?; tail -1 gpurun_out/t_zu.log; exit $rc
