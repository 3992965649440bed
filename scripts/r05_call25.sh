#!/bin/bash
# the commit queue's side rows at the headline shape (SPG_TRACE=3)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
SPG_TRACE=3 timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --extras none \
  > gpurun_out/b25.json 2> gpurun_out/b25.err || { tail -20 gpurun_out/b25.err; exit 1; }
grep "commit queue\|commit rows" gpurun_out/b25.err | tail -30
