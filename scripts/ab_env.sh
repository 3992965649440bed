#!/bin/bash
# A/B of one environment switch on the SNARK bench, alternating on the same box: ab_env.sh VAR "v1 v2" reps
# (AB_KERNEL=name1,name2 also prints those kernels' device ms per step from the bench line's kernel table)
VAR=$1; VALS=$2; REPS=${3:-3}
for r in $(seq $REPS); do
  for v in $VALS; do
    env $VAR=$v timeout -k 5 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/b_ab.json 2>/dev/null || exit $?
    echo "$VAR=$v $(python -c 'import json,os;d=json.load(open("gpurun_out/b_ab.json"));ks=[k for k in os.environ.get("AB_KERNEL","").split(",") if k];print(d["ms_per_step"], d.get("ms_per_step_median"), d.get("ms_per_step_min"), "dev", d.get("device_busy_ms_per_step"), *[(k, d["kernels"].get(k, {}).get("ms_per_step")) for k in ks])')"
  done
done
