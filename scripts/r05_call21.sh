#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
(cd scripts/micro && timeout -k 10 120 ./launch_cost > ../../gpurun_out/launch_cost.txt 2>&1) || exit 1
cat gpurun_out/launch_cost.txt
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29532 \
  bench.py --gpus 2 --backend gloo --steps 3 --warmup 1 --extras none > gpurun_out/b21_2ranks.json 2> gpurun_out/b21_2ranks.err \
  || { tail -20 gpurun_out/b21_2ranks.err; exit 1; }
wc -l gpurun_out/b21_2ranks.json
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_all.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests_all.log; exit $rc
