# more than 32 instances per R1CSProof: R1CS / SNARK / SPARK parity suites
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests/test_gpu_r1cs.py tests/test_gpu_snark.py tests/test_gpu_spark.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_t.log 2>&1; rc=$?; tail -5 gpurun_out/gpu_t.log; exit $rc
