#!/bin/bash
# Round 3: where SNARK::prove's 25 ms go -- host breakdown (SPG_TRACE=1, 2) and a kernel trace of 5 proves.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
SPG_TRACE=1 timeout -k 10 200 python scripts/trace_snark.py > gpurun_out/trace1.out 2> gpurun_out/trace1.err
rc=$?; grep -c "host breakdown" gpurun_out/trace1.err; [ $rc -eq 0 ] || exit $rc
SPG_TRACE=2 timeout -k 10 200 python scripts/trace_snark.py > gpurun_out/trace2.out 2> gpurun_out/trace2.err
rc=$?; [ $rc -eq 0 ] || exit $rc
SPG_TRACE=3 timeout -k 10 200 python scripts/trace_snark.py > gpurun_out/trace3.out 2> gpurun_out/trace3.err
rc=$?; [ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$R/gpurun_out/prof_snark" -o snark -- \
  python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --extras none > "$R/gpurun_out/snark_prof.json" 2> "$R/gpurun_out/snark_prof.err"
rc=$?; echo "prof rc=$rc"; exit $rc
