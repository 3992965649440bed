#!/bin/bash
# Round 3: host-pool knobs on the SNARK bench (slice size of host commitments, bucket-final chunks, workers)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export BENCH_ARGS="--extras none"
bash scripts/ab_env.sh SPG_SLICE_MIN "8 32 64" 3 || exit $?
bash scripts/ab_env.sh SPG_FINALS_K "4 2 8" 3 || exit $?
bash scripts/ab_env.sh SPG_POOL_THREADS "7 5 11" 2 || exit $?
