#!/bin/bash
# A/B of two libspg builds in ABBA order (drift over a session cancels in the pair differences):
#   ab_lib2.sh libA libB [blocks]   (paths relative to spartan-parallel_amd/; BENCH_ARGS, AB_STEPS)
A=$1; B=$2; N=${3:-3}
run() {
  SPG_LIB=$(pwd)/spartan-parallel_amd/$1 timeout -k 5 200 python bench.py --steps ${AB_STEPS:-20} --warmup 3 \
    --no-cpu-baseline --extras none ${BENCH_ARGS:-} > gpurun_out/b_ab2.json 2>/dev/null || exit $?
  python3 -c 'import json,sys;d=json.load(open("gpurun_out/b_ab2.json"));print(sys.argv[1], d["ms_per_step"], d.get("ms_per_step_median"), "dev", d.get("device_busy_ms_per_step"))' $1
}
for i in $(seq $N); do run $A; run $B; run $B; run $A; done
