#!/bin/bash
# A/B of one environment switch on the SNARK bench, alternating on the same box: ab_env.sh VAR "v1 v2" reps
VAR=$1; VALS=$2; REPS=${3:-3}
for r in $(seq $REPS); do
  for v in $VALS; do
    env $VAR=$v timeout -k 5 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/b_ab.json 2>/dev/null || exit $?
    echo "$VAR=$v $(python -c 'import json;d=json.load(open("gpurun_out/b_ab.json"));print(d["ms_per_step"], d.get("ms_per_step_median"), d.get("ms_per_step_min"))')"
  done
done
