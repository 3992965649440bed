#!/bin/bash
# Round 3: comb kernels with the next entry prefetched, wide comb at 4 windows per lane: parity, config-2 and SNARK A/B
# rows comb re-check through the SNARK golden tests
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_msm.py > gpurun_out/t_zh1.log 2>&1
rc=$?; tail -3 gpurun_out/t_zh1.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do for v in 0 1; do
SPG_COMB=$v timeout -k 10 200 python bench.py --workload msm --no-cpu-baseline > gpurun_out/b_zh.json 2> gpurun_out/b_zh.err || exit $?
python -c 'import json;d=json.load(open("gpurun_out/b_zh.json"));print("comb='$v'", d["ms_per_step"], d["ms_per_step_median"], "first", d.get("first_call_ms_incl_table_build"), "dev", d["valu_whole_msm"], d["result"][:16]); print({n:(v["ms_per_step"],v["launches_per_step"]) for n,v in d["kernels"].items()})'
done; done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_snark.py tests/test_gpu_r1cs.py tests/test_gpu_dropin.py > gpurun_out/t_zh.log 2>&1
rc=$?; tail -2 gpurun_out/t_zh.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 200 python bench.py --extras none --no-cpu-baseline > gpurun_out/b_zh2.json 2> gpurun_out/b_zh2.err || exit $?
python -c 'import json;d=json.load(open("gpurun_out/b_zh2.json"));print("snark", d["ms_per_step"], d["ms_per_step_median"], d["ms_per_step_min"], "busy", d["device_busy_ms_per_step"], d["proof_sha256"]); print({n:(v["ms_per_step"],v["launches_per_step"]) for n,v in d["kernels"].items() if "msm" in n})'
done
