#!/bin/bash
# Round 3: host fixed-base tables on huge pages (SPG_HOST_HUGE) x entry prefetch (SPG_HOST_PREFETCH): host-path Bullet
# proofs in situ (SPG_TRACE=3), SNARK bench; parity of the SNARK golden cases
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
cat /sys/kernel/mm/transparent_hugepage/enabled || true
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_snark.py > gpurun_out/t_zl.log 2>&1
rc=$?; tail -1 gpurun_out/t_zl.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for cfg in "0 0" "1 0" "1 3" "0 3"; do set -- $cfg
SPG_HOST_HUGE=$1 SPG_HOST_PREFETCH=$2 SPG_TRACE=3 TRACE_REPS=4 timeout -k 10 200 python3 scripts/trace_snark.py > /dev/null 2> gpurun_out/tr_zl.err || exit $?
python - "$1 $2" <<'PY'
import sys, re
L=[l for l in open('gpurun_out/tr_zl.err') if 'DotProductProofLog n=' in l or 'SNARK::prove host' in l]
idx=[i for i,l in enumerate(L) if 'SNARK::prove' in l]
tot=0; n=0
for i in range(1, len(idx)):
    for l in L[idx[i-1]+1:idx[i]]:
        if ' host:' in l:
            tot += float(re.search(r'total=(\d+)', l).group(1)); n += 1
snk=[float(re.search(r'total=(\d+)', L[i]).group(1)) for i in idx[1:]]
print('huge/pf', sys.argv[1], 'host proofs per prove', round(tot/(len(idx)-1)), 'us over', n//(len(idx)-1), 'proofs; prove', round(sum(snk)/len(snk)))
PY
done; done
for cfg in "0 0" "1 0"; do set -- $cfg
SPG_HOST_HUGE=$1 timeout -k 10 200 python bench.py --extras none --no-cpu-baseline > gpurun_out/b_zl.json 2> gpurun_out/b_zl.err || exit $?
python -c 'import json;d=json.load(open("gpurun_out/b_zl.json"));print("bench huge='$1'", d["ms_per_step"], d["ms_per_step_median"], d["ms_per_step_min"], d["proof_sha256"])'
done
