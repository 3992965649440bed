#!/bin/bash
# Round 3: wide comb (one large MSM, c = 8 byte windows, 25.8 GB at 2^16 generators): MSM parity, config-2 A/B,
# rows comb re-check through the SNARK golden tests
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_msm.py > gpurun_out/t_zg1.log 2>&1
rc=$?; tail -3 gpurun_out/t_zg1.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do for v in 0 1; do
SPG_COMB=$v timeout -k 10 200 python bench.py --workload msm --no-cpu-baseline > gpurun_out/b_zg.json 2> gpurun_out/b_zg.err || exit $?
python -c 'import json;d=json.load(open("gpurun_out/b_zg.json"));print("comb='$v'", d["ms_per_step"], d["ms_per_step_median"], "first", d.get("first_call_ms_incl_table_build"), "dev", d["valu_whole_msm"], d["result"][:16]); print({n:(v["ms_per_step"],v["launches_per_step"]) for n,v in d["kernels"].items()})'
done; done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_snark.py tests/test_gpu_r1cs.py tests/test_gpu_dropin.py > gpurun_out/t_zg.log 2>&1
rc=$?; tail -2 gpurun_out/t_zg.log; [ $rc -eq 0 ] || exit $rc
