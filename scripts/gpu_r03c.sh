#!/bin/bash
# Round 3: the config-2 MSM with phase probes, and its rocprofv3 kernel trace.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
SPG_BIG_PROBE=1 timeout -k 10 200 python bench.py --workload msm --steps 3 --warmup 1 --no-cpu-baseline \
  > gpurun_out/msm_probe.json 2> gpurun_out/msm_probe.err
rc=$?; grep "big " gpurun_out/msm_probe.err | tail -4; [ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_msm" -o msm -- \
  python3 "$R/bench.py" --workload msm --steps 10 --warmup 2 --no-cpu-baseline > "$R/gpurun_out/msm_prof.json" 2> "$R/gpurun_out/msm_prof.err"
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
f=$(find "$R/gpurun_out/prof_msm" -name '*kernel_stats.csv' | head -1); cut -d, -f1-6 "$f" | head -25
