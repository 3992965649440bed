#!/bin/bash
# tiny row commitments on the host pool: parity, trace, ABBA
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_msm.py \
  tests/test_gpu_snark.py tests/test_gpu_spark.py -k "golden or commit or tiny or oracle" > gpurun_out/t26.log 2>&1
rc=$?; tail -3 gpurun_out/t26.log; [ $rc = 0 ] || exit $rc
SPG_TRACE=3 timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --extras none \
  > gpurun_out/b26.json 2> gpurun_out/b26.err || { tail -20 gpurun_out/b26.err; exit 1; }
grep "commit rows" gpurun_out/b26.err | tail -8
bash scripts/ab_env2.sh SPG_HOST_COMMIT_MAX 0 1024 3 > gpurun_out/ab26.txt
cat gpurun_out/ab26.txt
