#!/bin/bash
# Round 3: large-MSM accumulation with one workgroup per bucket (looping over extra chunks) -- parity, bench, probes
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_msm.py > gpurun_out/t_msm.log 2>&1
rc=$?; tail -2 gpurun_out/t_msm.log; [ $rc -eq 0 ] || exit $rc
for k in 1 2; do
  timeout -k 10 200 python bench.py --workload msm --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/msm_v.json 2> gpurun_out/msm_v.err
  rc=$?; python3 -c "import json; d=json.load(open('gpurun_out/msm_v.json')); print(d['ms_per_step'], d['ms_per_step_median'], d.get('ms_per_step_incl_scalar_upload'), d['valu_whole_msm'], {k: v['ms_per_step'] for k, v in d['kernels'].items()})"; [ $rc -eq 0 ] || exit $rc
done
SPG_BIG_PROBE=1 timeout -k 10 200 python bench.py --workload msm --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/msm_probe.json 2> gpurun_out/msm_probe.err
rc=$?; grep "big accum" gpurun_out/msm_probe.err | tail -2; exit $rc
