#!/bin/bash
# Round 3: single-lane item accumulation of the large MSM -- parity, then items on/off and item length sweep,
# then the quad_madd throughput micro
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_msm.py \
  > gpurun_out/t_msm.log 2>&1
rc=$?; tail -2 gpurun_out/t_msm.log; [ $rc -eq 0 ] || exit $rc
for cfg in "0 0" "1 0" "0 0" "1 0"; do
  set -- $cfg
  SPG_BIG_ITEMS=$1 SPG_BIG_PF=$2 timeout -k 10 200 python bench.py --workload msm --steps 50 --warmup 5 --no-cpu-baseline \
    > gpurun_out/msm_v.json 2> gpurun_out/msm_v.err
  rc=$?; python3 -c "import json; d=json.load(open('gpurun_out/msm_v.json')); print('items=$1', d['ms_per_step'], d['ms_per_step_median'], d.get('ms_per_step_incl_scalar_upload'), d['valu_whole_msm'], {k: v['ms_per_step'] for k, v in d['kernels'].items()})"; [ $rc -eq 0 ] || exit $rc
done

