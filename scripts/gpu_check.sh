#!/bin/bash
# One GPU-box session: parity tests, bench, rocprofv3 kernel-trace summary. Stops at the first step that
# faults, aborts or times out (exit codes other than 0 / 1).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 ${T_TESTS:-600} python -m pytest tests -m gpu -q --maxfail=5 > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log; ok $rc || exit $rc
timeout -k 10 ${T_BENCH:-300} python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json; tail -5 gpurun_out/bench.err; [ $rc -eq 0 ] || exit $rc
if [ "${PROF:-1}" = "1" ]; then
  export TMPDIR=/tmp
  cd /tmp
  timeout -k 10 ${T_PROF:-300} rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o r1cs -- \
    python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$R/gpurun_out/prof_bench.json" 2> "$R/gpurun_out/prof.err"
  rc=$?; echo "prof rc=$rc"; tail -3 "$R/gpurun_out/prof.err"; [ $rc -eq 0 ] || exit $rc
  find "$R/gpurun_out/prof" -name '*stats*' | head
fi
