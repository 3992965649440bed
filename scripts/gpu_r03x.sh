#!/bin/bash
# Round 3: Cx MSM and Bullet round 0 launched together -- parity (SNARK / R1CS / SPARK / drop-in), A/B, trace
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_snark.py tests/test_gpu_r1cs.py tests/test_gpu_spark.py tests/test_gpu_dropin.py tests/test_gpu_verify.py > gpurun_out/t_ahead.log 2>&1
rc=$?; tail -2 gpurun_out/t_ahead.log; [ $rc -eq 0 ] || exit $rc
BENCH_ARGS="--extras none" bash scripts/ab_lib.sh lib/libspg_base.so lib/libspg.so 3 || exit $?
SPG_TRACE=2 timeout -k 10 200 python scripts/trace_snark.py > gpurun_out/trace2.out 2> gpurun_out/trace2.err || exit $?
grep "SNARK::prove host" gpurun_out/trace2.err | tail -1
