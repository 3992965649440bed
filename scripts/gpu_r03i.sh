#!/bin/bash
# Round 3: config-2 MSM after the launch fusion: parity, bench (twice), kernel trace
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_msm.py tests/test_gpu_dist.py -k "msm or failure or spark" > gpurun_out/t_msm.log 2>&1
rc=$?; tail -2 gpurun_out/t_msm.log; [ $rc -eq 0 ] || exit $rc
for k in 1 2; do
  timeout -k 10 200 python bench.py --workload msm --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/msm_v.json 2> gpurun_out/msm_v.err
  rc=$?; python3 -c "import json; d=json.load(open('gpurun_out/msm_v.json')); print(d['ms_per_step'], d['ms_per_step_median'], d.get('ms_per_step_incl_scalar_upload'), d['valu_whole_msm'], {k: v['ms_per_step'] for k, v in d['kernels'].items()})"; [ $rc -eq 0 ] || exit $rc
done
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_msm" -o msm -- \
  python3 "$R/bench.py" --workload msm --steps 20 --warmup 3 --no-cpu-baseline > "$R/gpurun_out/msm_prof.json" 2> "$R/gpurun_out/msm_prof.err"
rc=$?; echo "prof rc=$rc"; exit $rc
