#!/bin/bash
# A/B of two builds of libspg on the SNARK bench, alternating on the same box:
#   ab_lib.sh lib/libspg_base.so lib/libspg.so [reps]   (paths relative to spartan-parallel_amd/)
A=$1; B=$2; REPS=${3:-3}
for r in $(seq $REPS); do
  for L in $A $B; do
    SPG_LIB=$(pwd)/spartan-parallel_amd/$L timeout -k 5 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/b_ab.json 2>/dev/null || exit $?
    echo "$L $(python -c 'import json,os;d=json.load(open("gpurun_out/b_ab.json"));k=os.environ.get("AB_KERNEL");print(d["ms_per_step"], d.get("ms_per_step_median"), d.get("ms_per_step_min"), "dev", d.get("device_busy_ms_per_step"), k, d["kernels"].get(k, {}).get("ms_per_step") if k else "")')"
  done
done
