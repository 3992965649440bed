#!/bin/bash
# Round 3: glibc malloc trim / mmap thresholds (GLIBC_TUNABLES) on the SNARK bench
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
BIG=glibc.malloc.trim_threshold=1073741824:glibc.malloc.mmap_threshold=1073741824:glibc.malloc.top_pad=67108864
BENCH_ARGS="--extras none" bash scripts/ab_env.sh GLIBC_TUNABLES "glibc.malloc.check=0 $BIG" 4
