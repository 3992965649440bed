#!/bin/bash
# commit-queue batches: parity (goldens, forms, the checked two-stream build), flush laps, ABBA
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_snark.py \
  tests/test_gpu_large.py -k "golden or commit or tiny or oracle or checked or 2e20" > gpurun_out/t27.log 2>&1
rc=$?; tail -3 gpurun_out/t27.log; [ $rc = 0 ] || exit $rc
SPG_TRACE=2 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --extras none \
  > gpurun_out/b27.json 2> gpurun_out/b27.err || { tail -20 gpurun_out/b27.err; exit 1; }
grep "commit queue flush\|SNARK::prove host" gpurun_out/b27.err | tail -4
bash scripts/ab_env2.sh SPG_CQ_BATCH 0 1 3 > gpurun_out/ab27.txt
cat gpurun_out/ab27.txt
