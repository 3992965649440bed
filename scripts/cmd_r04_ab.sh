# same-box A/B of two builds of libspg (SPG_LIB), with the named kernels' device ms per step
L=$PWD/spartan-parallel_amd/lib
AB_KERNEL=${AB_KERNEL:-sc_phase1_fold_eval,sc_phase2_fold_eval,msm_bullet_round} bash scripts/ab_env.sh SPG_LIB "$L/libspg_prev.so $L/libspg.so" ${AB_REPS:-3}
