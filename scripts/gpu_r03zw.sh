#!/bin/bash
# Round 3: SPG_BULLET_HOST_MAX 32 (default) vs 64 after the host-table prefetch, 8 alternations of SPG_TRACE=1 totals
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
for r in 1 2 3 4 5 6 7 8; do for hm in 32 64; do
SPG_BULLET_HOST_MAX=$hm SPG_TRACE=1 TRACE_REPS=6 timeout -k 10 200 python3 scripts/trace_snark.py > /dev/null 2> gpurun_out/tr_zw.err || exit $?
python - "$hm" <<'PY'
import sys, re
v=[float(re.search(r'total=(\d+)', l).group(1)) for l in open('gpurun_out/tr_zw.err') if 'SNARK::prove host' in l][1:]
print(sys.argv[1], sorted(v)[len(v)//2])
PY
done; done
