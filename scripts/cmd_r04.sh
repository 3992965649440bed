L=$PWD/spartan-parallel_amd/lib
SPG_LIB=$L/libspg_lf.so timeout -k 10 400 python -u -m pytest tests/test_gpu_snark.py -x -q --timeout 200 --timeout-method thread > gpurun_out/lf_tests.log 2>&1 || { tail -20 gpurun_out/lf_tests.log; exit 1; }
tail -2 gpurun_out/lf_tests.log
AB_KERNEL=msm_bullet_round,sc_phase1_fold_eval bash scripts/ab_env.sh SPG_LIB "$L/libspg.so $L/libspg_lf.so" 3 || exit 1
bash scripts/ab_env.sh SPG_LAYER_PERSIST "0 1" 2 || exit 1
AB_KERNEL=msm_bullet_round bash scripts/ab_env.sh SPG_BCOMB_G "4 8" 2 || exit 1
