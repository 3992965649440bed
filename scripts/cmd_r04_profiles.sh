# kernel stats + PMC traffic of the single-GPU extras, each from its own workload run
for w in "msm:--workload msm" "rows:--workload rows" "r1cs22:--workload r1cs --config r1cs_2e22_p8" "spark24:--workload spark --log-nnz 24"; do
  tag=${w%%:*}; args=${w#*:}
  TAG=${tag}_ PROF=1 PMC=1 PROF_ARGS="$args" T_PROF=300 bash scripts/gpu_run.sh || exit 1
done
