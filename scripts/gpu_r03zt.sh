#!/bin/bash
# Round 3: config-2 MSM, LDS padding of the lane-form accumulation (caps workgroups per CU: 32 KB -> 5, 40 KB -> 4)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
for r in 1 2; do for pad in 0 8192 24576; do
SPG_BIG_LDS_PAD=$pad timeout -k 10 200 python bench.py --workload msm --no-cpu-baseline --steps 20 > gpurun_out/b_zt.json 2> gpurun_out/b_zt.err || exit $?
python -c 'import json;d=json.load(open("gpurun_out/b_zt.json"));print("pad='$pad'", d["ms_per_step"], d["ms_per_step_median"], d["valu_whole_msm"]["device_us_per_msm"], d["result"][:16], {n:v["ms_per_step"] for n,v in d["kernels"].items()})'
done; done
for pad in 0 8192; do
SPG_BIG_LDS_PAD=$pad SPG_BIG_PROBE=1 timeout -k 10 200 python bench.py --workload msm --no-cpu-baseline --steps 3 --warmup 1 > /dev/null 2> gpurun_out/probe_zt.err || exit $?
echo "pad=$pad $(grep 'big accum' gpurun_out/probe_zt.err | tail -1)"
done
