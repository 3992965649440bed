#!/bin/bash
# Round 3: batched polyeval bounds -- R1CS / SNARK / sharded parity, then A/B against HEAD with the SPG_TRACE=1 split
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_r1cs.py tests/test_gpu_snark.py tests/test_gpu_dropin.py tests/test_gpu_dist.py -k "not rccl_two" > gpurun_out/t_bound.log 2>&1
rc=$?; tail -2 gpurun_out/t_bound.log; [ $rc -eq 0 ] || exit $rc
BENCH_ARGS="--extras none" bash scripts/ab_lib.sh lib/libspg_base.so lib/libspg.so 3 || exit $?
SPG_TRACE=1 timeout -k 10 200 python scripts/trace_snark.py > gpurun_out/trace1.out 2> gpurun_out/trace1.err || exit $?
grep "R1CSProof::prove host" gpurun_out/trace1.err | tail -3
