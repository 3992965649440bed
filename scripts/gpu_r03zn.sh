#!/bin/bash
# Round 3 (late): the whole GPU suite, the default bench line, SPG_TRACE host breakdown, rocprof kernel stats + PMC passes
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -rs --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -4 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; tail -3 gpurun_out/bench.err; [ $rc -eq 0 ] || exit $rc
python -c 'import json;d=json.load(open("gpurun_out/bench.json"));print(d["ms_per_step"], d["ms_per_step_median"], d["ms_per_step_min"], d["device_busy_ms_per_step"], d["proof_bitexact_vs_cpu"]); print(d["config2_msm"]["ms_per_step_median"], d["config5_spark"]["ms_per_step_median"])'
SPG_TRACE=2 TRACE_REPS=4 timeout -k 10 200 python3 scripts/trace_snark.py > /dev/null 2> gpurun_out/host_breakdown.txt || exit $?
bash scripts/gpu_profile.sh
