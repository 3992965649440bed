#!/bin/bash
# Round 3: per-stream comb parts slot (the side stream's row commits raced the block-witness commit on one workspace
# slot): parity, then repeated bench steps (20 proves each must give the same bytes), A/B of window groups / host encodings
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_msm.py tests/test_gpu_snark.py tests/test_gpu_spark.py > gpurun_out/t_zp.log 2>&1
rc=$?; tail -1 gpurun_out/t_zp.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do for cfg in "4 384" "1 0"; do set -- $cfg
SPG_COMB_GMAX=$1 SPG_HOST_ENC_MAX=$2 timeout -k 10 200 python bench.py --extras none --no-cpu-baseline > gpurun_out/b_zp.json 2> gpurun_out/b_zp.err || exit $?
python -c 'import json;d=json.load(open("gpurun_out/b_zp.json"));print("bench '"$1 $2"'", d["ms_per_step"], d["ms_per_step_median"], d["ms_per_step_min"], d["device_busy_ms_per_step"], d["proof_sha256"])'
done; done
