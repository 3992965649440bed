#!/bin/bash
# A/B of one environment switch on the SNARK bench, printing per-step wall time and one kernel's device
# time per step (bench "kernels" entry): ab_kernel.sh VAR "v1 v2" reps kernel_scope
VAR=$1; VALS=$2; REPS=${3:-3}; K=$4
for r in $(seq $REPS); do
  for v in $VALS; do
    env $VAR=$v timeout -k 5 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/b_ab.json 2>/dev/null || exit $?
    echo "$VAR=$v $(python -c 'import json,sys;d=json.load(open("gpurun_out/b_ab.json"));k=d["kernels"].get(sys.argv[1],{});print(d["ms_per_step"], d.get("ms_per_step_median"), d.get("ms_per_step_min"), "dev", d["device_busy_ms_per_step"], sys.argv[1], k.get("ms_per_step"), k.get("launches_per_step"))' $K)"
  done
done
