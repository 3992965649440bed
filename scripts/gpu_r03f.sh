#!/bin/bash
# Round 3: large-MSM window sweep (c = 9, 10, 11), then the SNARK::prove trace pass (scripts/gpu_r03e.sh).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_msm.py -k "big or large or partial" \
  > gpurun_out/t_msm.log 2>&1
rc=$?; tail -2 gpurun_out/t_msm.log; [ $rc -eq 0 ] || exit $rc
for c in 9 10 11; do
  SPG_BIG_C=$c timeout -k 10 200 python bench.py --workload msm --steps 50 --warmup 5 --no-cpu-baseline \
    > gpurun_out/msm_v.json 2> gpurun_out/msm_v.err
  rc=$?; python3 -c "import json; d=json.load(open('gpurun_out/msm_v.json')); print('c=$c', d['ms_per_step'], d['ms_per_step_median'], d['valu_whole_msm'], {k: v['ms_per_step'] for k, v in d['kernels'].items()})"; [ $rc -eq 0 ] || exit $rc
done
bash scripts/gpu_r03e.sh
