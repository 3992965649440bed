#!/bin/bash
# Round 3: comb accumulation v2 (DPP lane join, row splits): parity, bench A/B of one row per workgroup vs 2048 workgroups
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_msm.py -k "commit_rows" > gpurun_out/t_zf1.log 2>&1
rc=$?; tail -3 gpurun_out/t_zf1.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_snark.py tests/test_gpu_msm.py tests/test_gpu_spark.py > gpurun_out/t_zf.log 2>&1
rc=$?; tail -2 gpurun_out/t_zf.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do for v in 1 2048; do
SPG_COMB_WGS=$v timeout -k 10 200 python bench.py --extras none --no-cpu-baseline > gpurun_out/b_zf.json 2> gpurun_out/b_zf.err || exit $?
python -c 'import json,sys;d=json.load(open("gpurun_out/b_zf.json"));print("wgs='$v'", d["ms_per_step"], d["ms_per_step_median"], d["ms_per_step_min"], "busy", d["device_busy_ms_per_step"], d["proof_sha256"]); k=d["kernels"]; print({n:(v["ms_per_step"],v["launches_per_step"]) for n,v in k.items() if "msm" in n})'
done; done
SPG_TRACE=1 TRACE_REPS=6 timeout -k 10 200 python3 scripts/trace_snark.py > /dev/null 2> gpurun_out/tr_zf.err || exit $?
python scripts/trace_avg.py gpurun_out/tr_zf.err input_commit block_sat block_eval pairwise perm_root perm_product shift io total
