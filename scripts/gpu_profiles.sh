# kernel stats + PMC traffic of the single-GPU extras (run as CMD of scripts/gpu_run.sh), each from its own workload run (nested gpu_run.sh calls
# with only the profiling steps: the outer call's TESTS / BENCH / CMD switches are cleared)
# PROFILE_WORKLOADS: "tag:bench args|tag:bench args|..."
IFS='|' read -r -a WL <<< "${PROFILE_WORKLOADS:-msm:--workload msm|rows:--workload rows|r1cs22:--workload r1cs --config r1cs_2e22_p8|spark24:--workload spark --log-nnz 24}"
for w in "${WL[@]}"; do
  tag=${w%%:*}; args=${w#*:}
  env -u TESTS -u BENCH -u CMD -u SMOKE TAG=${tag}_ PROF=1 PMC=1 PROF_ARGS="$args" T_PROF=300 bash scripts/gpu_run.sh || exit 1
done
if [ -n "${TRACE3:-}" ]; then  # per-proof Bullet / DotProductProofLog lines of one headline prove (SPG_TRACE=3)
  SPG_TRACE=3 TRACE_REPS=2 timeout -k 10 200 python scripts/trace_snark.py 2> gpurun_out/trace3.err > /dev/null || exit 1
fi
