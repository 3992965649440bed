# same-box A/Bs: comb workgroups of the block-witness row commit (headline), single-MSM comb vs buckets (config 2)
AB_KERNEL=msm_comb BENCH_ARGS="--extras none" bash scripts/ab_env.sh SPG_COMB_WGS "1024 2048 4096" 2 || exit 1
AB_KERNEL=msm_comb_single,msm_big_accum,msm_big_sort BENCH_ARGS="--workload msm" bash scripts/ab_env.sh SPG_BIG_COMB "0 1" 3 || exit 1
