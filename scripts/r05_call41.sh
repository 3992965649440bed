#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_msm.py tests/test_gpu_spark.py \
  tests/test_gpu_snark.py tests/test_gpu_r1cs.py -k "golden or commit or tiny or row_enc or oracle or comb" > gpurun_out/t41.log 2>&1
rc=$?; tail -2 gpurun_out/t41.log; [ $rc = 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --extras r1cs,msm,rows > gpurun_out/b41.json 2> gpurun_out/b41.err || exit 1
python3 scripts/bench_summary.py gpurun_out/b41.json
