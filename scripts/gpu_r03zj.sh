#!/bin/bash
# Round 3: device timeline + host laps after the comb commits and the shift bounds
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
export TMPDIR=/tmp
cd /tmp
SPG_TRACE=2 TRACE_REPS=6 timeout -k 10 200 python3 "$R/scripts/trace_snark.py" > /dev/null 2> "$R/gpurun_out/tr2b.err" || exit $?
echo "trace done"
TRACE_REPS=4 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$R/gpurun_out/tl2" -o tl -- \
  python3 "$R/scripts/trace_snark.py" > /dev/null 2> "$R/gpurun_out/tl.err" || exit $?
find "$R/gpurun_out/tl2" -name '*.csv'
