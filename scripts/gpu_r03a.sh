#!/bin/bash
# Round 3 quick check: MSM / drop-in / eq tests, the config-2 MSM bench, the madd-throughput micro.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v -s --timeout 240 --timeout-method thread tests/test_gpu_msm.py \
  tests/test_gpu_dropin.py tests/test_gpu_eq.py tests/test_gpu_dist.py::test_rccl_transport_one_rank > gpurun_out/t1.log 2>&1
rc=$?; tail -4 gpurun_out/t1.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --workload msm --steps 20 --warmup 3 > gpurun_out/msm.json 2> gpurun_out/msm.err
rc=$?; cat gpurun_out/msm.json; tail -3 gpurun_out/msm.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 60 ./scripts/micro/ext_throughput > gpurun_out/ext_throughput.txt
rc=$?; cat gpurun_out/ext_throughput.txt; exit $rc
