#!/bin/bash
# Round 3: per-commit times (SPG_TRACE=2 "commit rows=") with and without the latency-path comb / host encodings
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
for cfg in "4 384" "1 0" "4 0" "1 384"; do set -- $cfg
SPG_COMB_GMAX=$1 SPG_HOST_ENC_MAX=$2 SPG_TRACE=2 TRACE_REPS=4 timeout -k 10 200 python3 scripts/trace_snark.py > /dev/null 2> gpurun_out/tr_zq_$1_$2.err || exit $?
echo "== gmax/enc $1 $2"; grep "commit rows=" gpurun_out/tr_zq_$1_$2.err | tail -40 | sort | uniq -c | sort -rn | head -12
done
