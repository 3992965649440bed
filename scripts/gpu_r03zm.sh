#!/bin/bash
# Round 3: host-path Bullet proofs per prove (SPG_TRACE=3), huge pages x prefetch distance, 5 alternations
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
for r in 1 2 3 4 5; do for cfg in "0 0" "0 3" "1 3" "0 6" "1 0"; do set -- $cfg
SPG_HOST_HUGE=$1 SPG_HOST_PREFETCH=$2 SPG_TRACE=3 TRACE_REPS=5 timeout -k 10 200 python3 scripts/trace_snark.py > /dev/null 2> gpurun_out/tr_zm.err || exit $?
python - "$1 $2" <<'PY'
import sys, re
L=[l for l in open('gpurun_out/tr_zm.err') if 'DotProductProofLog n=' in l or 'SNARK::prove host' in l]
idx=[i for i,l in enumerate(L) if 'SNARK::prove' in l]
per=[]
for i in range(1, len(idx)):
    per.append(sum(float(re.search(r'total=(\d+)', l).group(1)) for l in L[idx[i-1]+1:idx[i]] if ' host:' in l))
snk=[float(re.search(r'total=(\d+)', L[i]).group(1)) for i in idx[1:]]
print('huge/pf', sys.argv[1], 'host proofs', sorted(per)[len(per)//2], 'prove', sorted(snk)[len(snk)//2])
PY
done; done
