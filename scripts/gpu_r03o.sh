#!/bin/bash
# Round 3: SNARK parity + A/B of host-side changes against HEAD's build
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_snark.py tests/test_gpu_dropin.py > gpurun_out/t_snark.log 2>&1
rc=$?; tail -2 gpurun_out/t_snark.log; [ $rc -eq 0 ] || exit $rc
bash scripts/ab_lib.sh lib/libspg_base.so lib/libspg.so 4
