#!/bin/bash
# Round 3: rows comb window width A/B (SPG_COMB_C 10 / 11 / 12: table 1.1 / 2.2 / 4.4 GB): parity per width, SNARK bench
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
for c in 10 11 12; do
SPG_COMB_C=$c timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_msm.py -k "commit_rows" > gpurun_out/t_zi$c.log 2>&1
rc=$?; echo "c=$c $(tail -1 gpurun_out/t_zi$c.log)"; [ $rc -eq 0 ] || exit $rc
done
for i in 1 2; do for c in 10 11 12; do
SPG_COMB_C=$c timeout -k 10 200 python bench.py --extras none --no-cpu-baseline > gpurun_out/b_zi.json 2> gpurun_out/b_zi.err || exit $?
python -c 'import json;d=json.load(open("gpurun_out/b_zi.json"));print("c='$c'", d["ms_per_step"], d["ms_per_step_median"], d["ms_per_step_min"], "busy", d["device_busy_ms_per_step"], d["proof_sha256"], {n:(v["ms_per_step"],v["madds_per_s"]) for n,v in d["kernels"].items() if "comb" in n})'
done; done
