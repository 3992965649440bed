#!/bin/bash
# Round 3: HIP API trace of SNARK::prove (which host calls wait, how many copies / launches per prove)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --stats --output-format csv -d "$R/gpurun_out/prof_api" -o api -- \
  python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --extras none > "$R/gpurun_out/api_prof.json" 2> "$R/gpurun_out/api_prof.err"
rc=$?; echo "prof rc=$rc"; ls "$R/gpurun_out/prof_api"; exit $rc
