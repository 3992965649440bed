#!/bin/bash
# Round 3: parity after the second-stream commit flush + interval-union busy time; a bench line
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_snark.py tests/test_gpu_msm.py tests/test_gpu_r1cs.py tests/test_gpu_spark.py tests/test_gpu_dropin.py > gpurun_out/t_zb.log 2>&1
rc=$?; tail -2 gpurun_out/t_zb.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 200 python bench.py --extras none --no-cpu-baseline > gpurun_out/b_zb.json 2> gpurun_out/b_zb.err || exit $?
python -c 'import json;d=json.load(open("gpurun_out/b_zb.json"));print(d["ms_per_step"], d["ms_per_step_median"], d["ms_per_step_min"], "busy", d["device_busy_ms_per_step"], "sum", round(sum(v["ms_per_step"] for v in d["kernels"].values()),3))'
done
