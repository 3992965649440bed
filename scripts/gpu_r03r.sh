#!/bin/bash
# Round 3: balanced work items in k_items -- parity, SNARK A/B against HEAD, config-5 SPARK
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
(cd scripts/micro && ARMED_ONLY=1 timeout -k 10 60 ./layer_phases > ../../gpurun_out/armed.txt 2>&1); cat gpurun_out/armed.txt
timeout -k 10 500 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_msm.py tests/test_gpu_snark.py tests/test_gpu_spark.py > gpurun_out/t_items.log 2>&1
rc=$?; tail -2 gpurun_out/t_items.log; [ $rc -eq 0 ] || exit $rc
AB_KERNEL=msm_bucket_items BENCH_ARGS="--extras none" bash scripts/ab_lib.sh lib/libspg_base.so lib/libspg.so 3 || exit $?
for L in lib/libspg_base.so lib/libspg.so; do
  SPG_LIB=$R/spartan-parallel_amd/$L timeout -k 10 300 python bench.py --workload spark --log-nnz 24 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/sp.json 2> gpurun_out/sp.err || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/sp.json'));print('spark $L', d['ms_per_step'], d['kernels']['msm_bucket_items'])"
done
