#!/bin/bash
# 13-bit comb windows by default: the comb-touching suites, then the bench line with config 2 / rows / config 4
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_msm.py tests/test_gpu_spark.py \
  tests/test_gpu_snark.py tests/test_gpu_r1cs.py tests/test_gpu_large.py -k "not 3x2e24" > gpurun_out/t48.log 2>&1
rc=$?; tail -2 gpurun_out/t48.log; [ $rc = 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --extras r1cs,msm,rows > gpurun_out/b48.json 2> gpurun_out/b48.err || exit 1
python3 scripts/bench_summary.py gpurun_out/b48.json
