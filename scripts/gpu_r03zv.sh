#!/bin/bash
# Round 3: knob re-check on the final tree (pool size, host Bullet threshold), SPG_TRACE=1 prove totals, 4 alternations
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null || true
for r in 1 2 3 4; do for cfg in "default" "SPG_POOL_THREADS=11" "SPG_POOL_THREADS=15" "SPG_BULLET_HOST_MAX=64" "SPG_HOST_PREFETCH=6"; do
if [ "$cfg" = default ]; then E=""; else E="$cfg"; fi
env $E SPG_TRACE=1 TRACE_REPS=6 timeout -k 10 200 python3 scripts/trace_snark.py > /dev/null 2> gpurun_out/tr_zv.err || exit $?
python - "$cfg" <<'PY'
import sys, re
v=[float(re.search(r'total=(\d+)', l).group(1)) for l in open('gpurun_out/tr_zv.err') if 'SNARK::prove host' in l][1:]
print(sys.argv[1], 'median', sorted(v)[len(v)//2], 'min', min(v))
PY
done; done
