#!/bin/bash
# Round 3 (final tree): the whole GPU suite and smoke(), then the config-2 / config-5 kernel stats + PMC passes
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -rs --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
bash scripts/gpu_r03y.sh
