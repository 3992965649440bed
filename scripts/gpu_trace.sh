# headline: host-time breakdown (SPG_TRACE=1), copy counts, then kernel stats and PMC traffic (gpu_run.sh PROF/PMC)
SPG_TRACE=1 TRACE_REPS=4 timeout -k 10 200 python scripts/trace_snark.py 2> gpurun_out/trace.err > /dev/null || exit 1
python scripts/trace_avg.py gpurun_out/trace.err input_commit block_sat block_eval pairwise perm_root perm_product shift io total
SPG_COPY_TRACE=1 TRACE_REPS=2 timeout -k 10 200 python scripts/trace_snark.py 2> gpurun_out/copies.err > /dev/null || exit 1
tail -40 gpurun_out/copies.err
