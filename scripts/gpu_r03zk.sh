#!/bin/bash
# Round 3: per-proof DotProductProofLog laps (SPG_TRACE=3) of the SNARK bench shape
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
SPG_TRACE=3 TRACE_REPS=4 timeout -k 10 200 python3 scripts/trace_snark.py > /dev/null 2> gpurun_out/tr3.err || exit $?
grep -c "DotProductProofLog n=" gpurun_out/tr3.err
