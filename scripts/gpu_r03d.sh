#!/bin/bash
# Round 3: large-MSM parity tests, then the config-2 MSM with phase probes and its timing.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_msm.py \
  > gpurun_out/t_msm.log 2>&1
rc=$?; tail -3 gpurun_out/t_msm.log; [ $rc -eq 0 ] || exit $rc
for f in 2 1; do
  SPG_BIG_ACC=$f SPG_BIG_PROBE=1 timeout -k 10 200 python bench.py --workload msm --steps 3 --warmup 1 --no-cpu-baseline \
    > gpurun_out/msm_probe$f.json 2> gpurun_out/msm_probe$f.err
  rc=$?; echo "form $f"; grep "big " gpurun_out/msm_probe$f.err | tail -2; [ $rc -eq 0 ] || exit $rc
done
for v in "SPG_BIG_ACC=2" "SPG_BIG_ACC=1" "SPG_BIG_ACC=2 SPG_BIG_C=11" "SPG_BIG_ACC=1 SPG_BIG_C=11"; do
  env $v timeout -k 10 200 python bench.py --workload msm --steps 50 --warmup 5 --no-cpu-baseline \
    > gpurun_out/msm_v.json 2> gpurun_out/msm_v.err
  rc=$?; python3 -c "import json; d=json.load(open('gpurun_out/msm_v.json')); print('$v', d['ms_per_step'], d['ms_per_step_median'], d['valu_whole_msm'], {k: v['ms_per_step'] for k, v in d['kernels'].items()})"; [ $rc -eq 0 ] || exit $rc
done
