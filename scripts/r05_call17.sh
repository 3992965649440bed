#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
T=600 bash scripts/session_r05.sh tests "test_gpu_r1cs or test_config4 or test_snark_2e20_headline or test_gpu_snark" || exit 1
for i in 1 2; do
  timeout -k 10 300 python bench.py --workload r1cs --config r1cs_2e22_p8 --no-cpu-baseline > gpurun_out/b17_r1cs.json 2>/dev/null || exit 1
  python3 -c 'import json;d=json.load(open("gpurun_out/b17_r1cs.json"));print("r1cs", d["ms_per_step"], d["ms_per_step_median"], d["device_busy_ms_per_step"])'
  timeout -k 10 300 python bench.py --no-cpu-baseline --extras none > gpurun_out/b17_snark.json 2>/dev/null || exit 1
  python3 -c 'import json;d=json.load(open("gpurun_out/b17_snark.json"));print("snark", d["ms_per_step"], d["ms_per_step_median"], d["device_busy_ms_per_step"])'
done
