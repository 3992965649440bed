#!/bin/bash
# Round 3: PMC HBM traffic (FETCH_SIZE, WRITE_SIZE passes) + kernel stats of the config-2 MSM and config-5 SPARK
# workloads, each in its own runs, so bench.py reports every workload's traffic from its own launches
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
export TMPDIR=/tmp
cd /tmp
for W in "msm_2e16:--workload msm --log-msm 16 --steps 5 --warmup 1" "spark_2e24:--workload spark --log-nnz 24 --mode replicas --steps 2 --warmup 1"; do
  N=${W%%:*}; BA="${W#*:} --no-cpu-baseline"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$N" -o k -- \
    python3 "$R/bench.py" $BA > "$R/gpurun_out/prof_$N.json" 2> "$R/gpurun_out/prof_$N.err" || exit $?
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/pmcf_$N" -o f -- \
    python3 "$R/bench.py" $BA > /dev/null 2> "$R/gpurun_out/pmcf_$N.err" || exit $?
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/pmcw_$N" -o w -- \
    python3 "$R/bench.py" $BA > /dev/null 2> "$R/gpurun_out/pmcw_$N.err" || exit $?
  python3 "$R/scripts/pmc_traffic.py" "$R/gpurun_out/pmcf_$N" "$R/gpurun_out/pmcw_$N" "$R/gpurun_out/pmc_traffic_$N.json" > /dev/null
  echo "$N done"
done
