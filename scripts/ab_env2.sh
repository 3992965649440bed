#!/bin/bash
# A/B of one environment switch in ABBA order on the current build:
#   ab_env2.sh VAR valA valB [blocks]   (BENCH_ARGS, AB_STEPS)
V=$1; A=$2; B=$3; N=${4:-3}
run() {
  env $V=$1 timeout -k 5 200 python bench.py --steps ${AB_STEPS:-20} --warmup 3 --no-cpu-baseline --extras none \
    ${BENCH_ARGS:-} > gpurun_out/b_ae2.json 2>/dev/null || exit $?
  python3 -c 'import json,sys;d=json.load(open("gpurun_out/b_ae2.json"));r=d.get("roofline") or {};print(sys.argv[1], d["ms_per_step"], d.get("ms_per_step_median"), "dev", d.get("device_busy_ms_per_step"), r.get("kernel"), r.get("avg_launch_us"), r.get("frac"))' "$V=$1"
}
for i in $(seq $N); do run $A; run $B; run $B; run $A; done
