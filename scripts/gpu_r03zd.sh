#!/bin/bash
# Round 3: shift/perm-product/IO bounds in one burst + host table prefetch: host micro A/B, SNARK parity, bench A/B
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
g++ -O2 -std=c++17 -march=x86-64-v3 -pthread -I spartan-parallel_amd/csrc -I include scripts/micro/host_ops.cpp -o /tmp/host_ops || exit 1
for r in 1 2 3; do for v in 0 4; do echo -n "pf=$v "; SPG_HOST_PREFETCH=$v timeout -k 5 60 taskset -c 0-7 /tmp/host_ops | grep -E "Bullet round|commit_many 3" | tr '\n' ' '; echo; done; done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_snark.py tests/test_gpu_dropin.py > gpurun_out/t_zd.log 2>&1
rc=$?; tail -2 gpurun_out/t_zd.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do for v in 0 4; do
SPG_HOST_PREFETCH=$v timeout -k 10 200 python bench.py --extras none --no-cpu-baseline > gpurun_out/b_zd.json 2> gpurun_out/b_zd.err || exit $?
python -c 'import json,sys;d=json.load(open("gpurun_out/b_zd.json"));print("pf='$v'", d["ms_per_step"], d["ms_per_step_median"], d["ms_per_step_min"], "busy", d["device_busy_ms_per_step"], d["proof_sha256"])'
done; done
SPG_TRACE=1 TRACE_REPS=6 timeout -k 10 200 python3 scripts/trace_snark.py > /dev/null 2> gpurun_out/tr_zd.err || exit $?
python scripts/trace_avg.py gpurun_out/tr_zd.err input_commit block_sat block_eval pairwise perm_root perm_product shift io total
