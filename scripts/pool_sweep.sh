#!/bin/bash
# SNARK bench under host-pool settings (threads, spin microseconds): one line each
CFG=("15 300" "15 0" "11 300" "7 300" "11 100" "7 0")
[ -n "${CFGS:-}" ] && IFS=, read -ra CFG <<< "$CFGS"
for cfg in "${CFG[@]}"; do
  set -- $cfg
  SPG_POOL_THREADS=$1 SPG_POOL_SPIN_US=$2 timeout -k 5 120 python bench.py --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline \
    > gpurun_out/b_pool.json 2>/dev/null || exit $?
  echo "threads=$1 spin=$2 $(python -c 'import json;d=json.load(open("gpurun_out/b_pool.json"));print(d["ms_per_step"])')"
done
