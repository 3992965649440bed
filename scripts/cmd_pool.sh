# fused R1CS folds: parity tests, then A/B against the previous build (mean / median / min ms per prove)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_r1cs.py tests/test_gpu_snark.py tests/test_gpu_dist.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_t.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_t.log; [ $rc -eq 0 ] || exit $rc
bash scripts/ab_lib.sh lib/libspg_base.so lib/libspg.so 4
