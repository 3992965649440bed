#!/bin/bash
# round-5 GPU call: SNARK parity of the new build, library A/B (Bullet R = 2 + sat_prove staging vs the previous
# build), config 5 in-process after the headline with and without the other extras
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
T=400 bash scripts/session_r05.sh tests "test_gpu_snark and not round_forms" || exit 1
timeout -k 10 700 bash scripts/ab_lib.sh lib/libspg_prev.so lib/libspg.so 3 > gpurun_out/ab_lib4.txt 2>&1 || { cat gpurun_out/ab_lib4.txt; exit 1; }
cat gpurun_out/ab_lib4.txt
timeout -k 10 400 python bench.py --steps 10 --warmup 2 --extras spark --no-cpu-baseline > gpurun_out/b4_spark.json 2> gpurun_out/b4_spark.err || exit 1
python3 -c 'import json;d=json.load(open("gpurun_out/b4_spark.json"));c=d["config5_spark"];print("spark after headline", d["ms_per_step"], c["ms_per_step"], c["ms_per_step_median"], c["device_busy_ms_per_step"])'
timeout -k 10 600 python bench.py --steps 10 --warmup 2 --extras r1cs,spark > gpurun_out/b4_r1cs_spark.json 2> gpurun_out/b4_r1cs_spark.err || exit 1
python3 -c 'import json;d=json.load(open("gpurun_out/b4_r1cs_spark.json"));c=d["config5_spark"];r=d["config4_r1cs"];print("r1cs+spark with cpu", d["ms_per_step"], r["ms_per_step"], r["device_busy_ms_per_step"], c["ms_per_step"], c["ms_per_step_median"], c["device_busy_ms_per_step"])'
