# same-box A/Bs: the previous build against this one (SPG_LIB), then the host-path Bullet threshold
L=$PWD/spartan-parallel_amd/lib
AB_KERNEL=sc_phase1_fold_eval,spark_layer_round,msm_bullet_round bash scripts/ab_env.sh SPG_LIB "$L/libspg_prev.so $L/libspg.so" 3 || exit 1
AB_KERNEL=msm_bullet_round bash scripts/ab_env.sh SPG_BULLET_HOST_MAX "0 8 32" 2 || exit 1
