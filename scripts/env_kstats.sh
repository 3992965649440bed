#!/bin/bash
# rocprofv3 kernel stats of a short bench run per value of one environment variable:
#   VAR=SPG_FINAL_SL VALS="128 64 32" bash scripts/env_kstats.sh   -> gpurun_out/kstats_<val>/k_kernel_stats.csv
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp; export TMPDIR=/tmp
for v in $VALS; do
  env "$VAR=$v" true  # validate
  export "$VAR=$v"
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/kstats_$v" -o k -- \
    python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > "$R/gpurun_out/kstats_$v.json" 2>/dev/null
done
