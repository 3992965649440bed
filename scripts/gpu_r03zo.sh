#!/bin/bash
# Round 3: latency-path row commits through the comb (window groups per scalar for few rows) + host encodings of
# small point batches: parity, then SNARK bench / trace A/B
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_msm.py tests/test_gpu_snark.py tests/test_gpu_spark.py tests/test_gpu_dropin.py tests/test_gpu_dist.py > gpurun_out/t_zo.log 2>&1
rc=$?; tail -2 gpurun_out/t_zo.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do for cfg in "4 384" "1 0" "4 0" "1 384"; do set -- $cfg
SPG_COMB_GMAX=$1 SPG_HOST_ENC_MAX=$2 SPG_TRACE=1 TRACE_REPS=5 timeout -k 10 200 python3 scripts/trace_snark.py > /dev/null 2> gpurun_out/tr_zo.err || exit $?
echo "gmax/enc $1 $2 $(python scripts/trace_avg.py gpurun_out/tr_zo.err input_commit block_eval pairwise perm_root total)"
done; done
for cfg in "1 0" "4 384" "1 0" "4 384"; do set -- $cfg
SPG_COMB_GMAX=$1 SPG_HOST_ENC_MAX=$2 timeout -k 10 200 python bench.py --extras none --no-cpu-baseline > gpurun_out/b_zo.json 2> gpurun_out/b_zo.err || exit $?
python -c 'import json;d=json.load(open("gpurun_out/b_zo.json"));print("bench '"$1 $2"'", d["ms_per_step"], d["ms_per_step_median"], d["ms_per_step_min"], d["device_busy_ms_per_step"], d["proof_sha256"])'
done
