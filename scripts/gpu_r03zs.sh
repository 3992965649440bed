#!/bin/bash
# Round 3: config-2 MSM, workgroup count of the lane-form accumulation (SPG_BIG_GRID) and the phase probe
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
for r in 1 2; do for g in 0 512 768 256; do
if [ $g = 0 ]; then unset SPG_BIG_GRID; else export SPG_BIG_GRID=$g; fi
timeout -k 10 200 python bench.py --workload msm --no-cpu-baseline --steps 20 > gpurun_out/b_zs.json 2> gpurun_out/b_zs.err || exit $?
python -c 'import json;d=json.load(open("gpurun_out/b_zs.json"));print("grid='$g'", d["ms_per_step"], d["ms_per_step_median"], d["valu_whole_msm"]["device_us_per_msm"], d["result"][:16], {n:v["ms_per_step"] for n,v in d["kernels"].items()})'
done; done
unset SPG_BIG_GRID
SPG_BIG_PROBE=1 timeout -k 10 200 python bench.py --workload msm --no-cpu-baseline --steps 3 --warmup 1 > /dev/null 2> gpurun_out/probe_zs.err || exit $?
grep "big accum\|blockIdx" gpurun_out/probe_zs.err | tail -10
