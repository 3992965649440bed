#!/bin/bash
# single MSM on the comb by default: the MSM suite, and the config-2 line
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_msm.py tests/test_gpu_dist.py \
  > gpurun_out/t33.log 2>&1
rc=$?; tail -3 gpurun_out/t33.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --extras msm > gpurun_out/b33.json 2> gpurun_out/b33.err \
  || { tail -5 gpurun_out/b33.err; exit 1; }
python3 -c 'import json;d=json.load(open("gpurun_out/b33.json"))["config2_msm"];print(d["ms_per_step"], d.get("ms_per_step_median"), d["roofline"]["kernel"], d["roofline"]["frac"], {k:v["ms_per_step"] for k,v in d["kernels"].items()})'
