#!/bin/bash
# Round 3 (final tree): one more default bench line (all extras, CPU baselines)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
uptime
timeout -k 10 500 python bench.py > gpurun_out/bench_b.json 2> gpurun_out/bench_b.err
rc=$?; tail -2 gpurun_out/bench_b.err; [ $rc -eq 0 ] || exit $rc
python -c 'import json;d=json.load(open("gpurun_out/bench_b.json"));print(d["ms_per_step"], d["ms_per_step_median"], d["ms_per_step_min"], d["device_busy_ms_per_step"], d["proof_bitexact_vs_cpu"], d["config2_msm"]["ms_per_step_median"], d["config5_spark"]["ms_per_step_median"])'
