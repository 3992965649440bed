#!/bin/bash
# The same-box A/B sets of round 4, by name: ab_sets.sh NAME [NAME ...]. Each runs scripts/ab_env.sh
# (alternating bench runs of one switch) with the kernels whose device ms per step it prints. `build` compares the
# previous build of the library (spartan-parallel_amd/lib/libspg_prev.so, built from the commit before) with this one.
L=$PWD/spartan-parallel_amd/lib
export BENCH_ARGS=${BENCH_ARGS:---extras none}
for set in "$@"; do
  case $set in
    persist) bash scripts/ab_env.sh SPG_LAYER_PERSIST "0 1" 3 ;;
    fuse) bash scripts/ab_env.sh SPG_SC_FUSE "0 1" 2 ;;
    bcomb) AB_KERNEL=msm_bullet_round bash scripts/ab_env.sh SPG_BULLET_COMB "0 1" 2 ;;
    bshape) AB_KERNEL=msm_bullet_round bash scripts/ab_env.sh SPG_BCOMB_R "4 8 16" 2 &&
            AB_KERNEL=msm_bullet_round bash scripts/ab_env.sh SPG_BCOMB_G "8 11" 2 ;;
    bbs) AB_KERNEL=msm_bullet_round bash scripts/ab_env.sh SPG_BCOMB_BS "0 64 128" 2 ;;
    bhost) AB_KERNEL=msm_bullet_round bash scripts/ab_env.sh SPG_BULLET_HOST_MAX "0 8 32" 2 ;;
    build) AB_KERNEL=${AB_KERNEL:-sc_phase1_fold_eval,sc_phase2_fold_eval,spark_layer_round,msm_bullet_round} \
             bash scripts/ab_env.sh SPG_LIB "$L/libspg_prev.so $L/libspg.so" ${AB_REPS:-3} ;;
    zside) AB_KERNEL=z_fill,spmv_block,sc_phase1_fold_eval bash scripts/ab_env.sh SPG_Z_SIDE "0 1" ${AB_REPS:-3} ;;
    # rocprof kernel stats of the previous build, this build, and this build with the Z fill in order (spmv launch time)
    spmvprof) P="env -u TESTS -u BENCH -u CMD -u SMOKE -u PMC PROF=1 T_PROF=200"
              $P SPG_LIB=$L/libspg_prev.so TAG=spA_ bash scripts/gpu_run.sh && $P TAG=spB_ bash scripts/gpu_run.sh &&
              $P SPG_Z_SIDE=0 TAG=spC_ bash scripts/gpu_run.sh ;;
    zafter) AB_KERNEL=sc_phase1_fold_eval bash scripts/ab_env.sh SPG_Z_AFTER "0 2 4" 2 ;;
    zlateprof) env -u TESTS -u BENCH -u CMD -u SMOKE -u PMC PROF=1 T_PROF=200 TAG=spD_ bash scripts/gpu_run.sh ;;
    combwgs) AB_KERNEL=msm_comb bash scripts/ab_env.sh SPG_COMB_WGS "1024 2048 4096" 2 ;;
    bigcomb) AB_KERNEL=msm_comb_single,msm_big_accum,msm_big_sort BENCH_ARGS="--workload msm" \
               bash scripts/ab_env.sh SPG_BIG_COMB "0 1" 3 ;;
    spark24) timeout -k 10 300 python bench.py --workload spark --log-nnz 24 --steps 5 --warmup 1 --no-cpu-baseline \
               > gpurun_out/spark24.json 2> gpurun_out/spark24.err &&
             python3 scripts/bench_summary.py gpurun_out/spark24.json ;;
    *) echo "unknown set $set"; exit 2 ;;
  esac || exit $?
done
