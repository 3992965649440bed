#!/bin/bash
# A/B of whole environment configurations on the SNARK bench, alternating on one box:
#   ab_confs.sh reps "CONF1" "CONF2" ...   (a CONF is a space-separated list of VAR=value, "-" for the defaults)
# prints per run: mean / median / fastest ms per prove, device busy, and (AB_KERNEL=a,b) those kernels' ms per prove
REPS=$1; shift
for r in $(seq $REPS); do
  for c in "$@"; do
    E=(); [ "$c" != "-" ] && read -ra E <<< "$c"
    env "${E[@]}" timeout -k 5 150 python bench.py --steps ${AB_STEPS:-20} --warmup 3 --no-cpu-baseline --extras none \
      > gpurun_out/b_ab.json 2>/dev/null || exit $?
    echo "[$c] $(python -c 'import json,os;d=json.load(open("gpurun_out/b_ab.json"));ks=[k for k in os.environ.get("AB_KERNEL","").split(",") if k];print(d["ms_per_step"], d.get("ms_per_step_median"), d.get("ms_per_step_min"), "dev", d.get("device_busy_ms_per_step"), *[(k, d["kernels"].get(k, {}).get("ms_per_step")) for k in ks])')"
  done
done
