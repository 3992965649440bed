# SNARK with more than 32 block types: GPU proof vs the oracle
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_snark.py -x -q -k "large" --timeout 300 --timeout-method thread > gpurun_out/gpu_t.log 2>&1; rc=$?; tail -15 gpurun_out/gpu_t.log; exit $rc
