# Bullet comb round shapes (workgroup points R, window groups G) and config 5 with the default build
AB_KERNEL=msm_bullet_round bash scripts/ab_env.sh SPG_BCOMB_R "4 8 16" 2 || exit 1
AB_KERNEL=msm_bullet_round bash scripts/ab_env.sh SPG_BCOMB_G "8 11" 2 || exit 1
timeout -k 10 300 python bench.py --workload spark --log-nnz 24 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/spark24.json 2> gpurun_out/spark24.err || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/spark24.json'));print('spark24', d['ms_per_step'], d.get('ms_per_step_median'), {k:v['ms_per_step'] for k,v in list(d['kernels'].items())[:8]})"
