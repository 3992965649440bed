#!/bin/bash
# Round 3: three default-length SNARK bench runs with per-step laps (box noise vs the tree)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null || true; uptime
for i in 1 2 3; do
timeout -k 10 200 python bench.py --extras none --no-cpu-baseline > gpurun_out/b_zr$i.json 2> gpurun_out/b_zr.err || exit $?
python -c 'import json;d=json.load(open("gpurun_out/b_zr'$i'.json"));print(d["ms_per_step"], d["ms_per_step_median"], d["ms_per_step_min"], d["device_busy_ms_per_step"], d["ms_per_step_laps"])'
done
