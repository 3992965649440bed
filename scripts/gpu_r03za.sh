#!/bin/bash
# Round 3: SPG_CQ_SIDE 0/1 alternated, SPG_TRACE=1 means over 7 proves per run
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
for r in 1 2 3 4; do
  for v in 0 1; do
    SPG_CQ_SIDE=$v SPG_TRACE=1 TRACE_REPS=8 timeout -k 10 200 python scripts/trace_snark.py > /dev/null 2> gpurun_out/tr_s$v.err || exit $?
    echo "SIDE=$v $(python scripts/trace_avg.py gpurun_out/tr_s$v.err input_commit block_sat block_eval pairwise total)"
  done
done
