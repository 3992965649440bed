#!/bin/bash
# rocprofv3 kernel-trace stats (csv) + two PMC passes (FETCH_SIZE, WRITE_SIZE) of a short bench run.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
export TMPDIR=/tmp
cd /tmp
BA="--steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:---extras none}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o bench -- \
  python3 "$R/bench.py" $BA > "$R/gpurun_out/prof_bench.json" 2> "$R/gpurun_out/prof.err" || exit $?
echo "stats done"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/pmc_fetch" -o f -- \
  python3 "$R/bench.py" $BA > /dev/null 2> "$R/gpurun_out/pmc_fetch.err" || exit $?
echo "fetch done"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/pmc_write" -o w -- \
  python3 "$R/bench.py" $BA > /dev/null 2> "$R/gpurun_out/pmc_write.err" || exit $?
echo "write done"
python3 "$R/scripts/pmc_traffic.py" "$R/gpurun_out/pmc_fetch" "$R/gpurun_out/pmc_write" "$R/gpurun_out/pmc_traffic.json"
find "$R/gpurun_out/prof" -name '*.csv'
