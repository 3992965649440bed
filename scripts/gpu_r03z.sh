#!/bin/bash
# Round 3: latency-path witness commits on the second stream beside the early block_vars MSM -- parity, A/B, trace;
# batch-MSM item size / segment width sweeps
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_snark.py tests/test_gpu_dropin.py tests/test_gpu_verify.py > gpurun_out/t_side.log 2>&1
rc=$?; tail -2 gpurun_out/t_side.log; [ $rc -eq 0 ] || exit $rc
SPG_ITEM_K=32 SPG_SEG_M=4 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_snark.py tests/test_gpu_msm.py::test_commit_rows tests/test_gpu_msm.py::test_commit_rows_wide > gpurun_out/t_itemk.log 2>&1
rc=$?; tail -2 gpurun_out/t_itemk.log; [ $rc -eq 0 ] || exit $rc
export BENCH_ARGS="--extras none"
bash scripts/ab_env.sh SPG_CQ_SIDE "0 1" 3 || exit $?
export AB_KERNEL=msm_bucket_items,msm_segments,msm_final
bash scripts/ab_env.sh SPG_ITEM_K "16 24 32" 2 || exit $?
bash scripts/ab_env.sh SPG_SEG_M "8 4 16" 2 || exit $?
for v in 0 1; do
  SPG_CQ_SIDE=$v SPG_TRACE=2 timeout -k 10 200 python scripts/trace_snark.py > gpurun_out/trace_side$v.out 2> gpurun_out/trace_side$v.err || exit $?
  echo "SPG_CQ_SIDE=$v"; grep "commit queue flush" gpurun_out/trace_side$v.err | tail -2; grep "SNARK::prove host" gpurun_out/trace_side$v.err | tail -1
done
