#!/bin/bash
# One GPU-box session, parameterised by environment (replaces the per-run scripts of rounds 1-3):
#   TESTS=1     pytest -m gpu (PYTEST_K: -k filter; T_TESTS: time limit, default 900 s)
#   SMOKE=1     __graft_entry__.smoke()
#   BENCH=1     python bench.py $BENCH_ARGS > gpurun_out/${TAG}bench.json (T_BENCH, default 600 s)
#   PROF=1      rocprofv3 --kernel-trace --stats of bench.py $PROF_ARGS (csv under gpurun_out/${TAG}prof)
#   PMC=1       two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) of bench.py $PROF_ARGS -> ${TAG}pmc_traffic.json
#   TRACE=hipt  kernel + HIP runtime API + memory-copy trace of traced proves (scripts/trace_snark.py), lap events in
#               gpurun_out/${TAG}kt.err (csv under gpurun_out/${TAG}kt)
#   TRACE=gaps  kernel trace + host lap events of 6 proves -> per-prove idle gaps by transition and by host lap
#               (scripts/kernel_gaps.py -> gpurun_out/${TAG}kt_gaps.txt; MARK: the kernel that opens a prove)
#   AB="VAR 'v1 v2' n"  traced same-box A/B of one switch (scripts/ab_trace.sh)
#   CMD="..."   one extra command, run last under its own time limit (T_CMD, default 300 s)
# Every step runs under its own `timeout -k 10`; the session stops at the first failing step.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${TAG:-}
uptime
if [ "${TESTS:-0}" = "1" ]; then
  K=()
  [ -n "${PYTEST_K:-}" ] && K=(-k "$PYTEST_K")
  timeout -k 10 ${T_TESTS:-900} python -u -m pytest tests -m gpu -x -v --timeout ${T_TEST1:-300} \
    --timeout-method thread "${K[@]}" > gpurun_out/${TAG}gpu_tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/${TAG}gpu_tests.log; [ $rc -eq 0 ] || exit $rc
fi
if [ "${SMOKE:-0}" = "1" ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/${TAG}smoke.log; [ $rc -eq 0 ] || exit $rc
fi
if [ "${BENCH:-0}" = "1" ]; then
  timeout -k 10 ${T_BENCH:-600} python bench.py ${BENCH_ARGS:-} > gpurun_out/${TAG}bench.json 2> gpurun_out/${TAG}bench.err
  rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/${TAG}bench.err; [ $rc -eq 0 ] || exit $rc
  python3 scripts/bench_summary.py gpurun_out/${TAG}bench.json || true
fi
PA="--steps 3 --warmup 1 --no-cpu-baseline ${PROF_ARGS:---extras none}"
if [ "${PROF:-0}" = "1" ]; then
  export TMPDIR=/tmp
  (cd /tmp && timeout -k 10 ${T_PROF:-400} rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/${TAG}prof" \
    -o prof -- python3 "$R/bench.py" $PA > "$R/gpurun_out/${TAG}prof_bench.json" 2> "$R/gpurun_out/${TAG}prof.err")
  rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$R/gpurun_out/${TAG}prof.err"; exit $rc; }
fi
if [ "${PMC:-0}" = "1" ]; then
  export TMPDIR=/tmp
  (cd /tmp && timeout -k 10 ${T_PROF:-400} rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/${TAG}pmc_fetch" \
    -o f -- python3 "$R/bench.py" $PA > /dev/null 2> "$R/gpurun_out/${TAG}pmc_fetch.err")
  rc=$?; echo "pmc fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
  (cd /tmp && timeout -k 10 ${T_PROF:-400} rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/${TAG}pmc_write" \
    -o w -- python3 "$R/bench.py" $PA > /dev/null 2> "$R/gpurun_out/${TAG}pmc_write.err")
  rc=$?; echo "pmc write rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 scripts/pmc_traffic.py "$R/gpurun_out/${TAG}pmc_fetch" "$R/gpurun_out/${TAG}pmc_write" \
    "$R/gpurun_out/${TAG}pmc_traffic.json"
fi
if [ -n "${TRACE:-}" ]; then
  export TMPDIR=/tmp
  if [ "$TRACE" = "hipt" ]; then
    (cd /tmp && SPG_TRACE=2 SPG_TRACE_EVENTS=1 TRACE_REPS=4 timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace \
      --memory-copy-trace --output-format csv -d "$R/gpurun_out/${TAG}kt" -o kt -- python3 "$R/scripts/trace_snark.py" \
      > /dev/null 2> "$R/gpurun_out/${TAG}kt.err")
    rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
  else
    (cd /tmp && SPG_TRACE=2 SPG_TRACE_EVENTS=1 TRACE_REPS=6 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv \
      -d "$R/gpurun_out/${TAG}kt" -o kt -- python3 "$R/scripts/trace_snark.py" > /dev/null 2> "$R/gpurun_out/${TAG}kt.err")
    rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
    MARK="${MARK:-k_comb_accum<13, 1>}" SKIP=1 python3 scripts/kernel_gaps.py gpurun_out/${TAG}kt XX > gpurun_out/${TAG}kt_gaps.txt
    MARK="${MARK:-k_comb_accum<13, 1>}" SKIP=1 EVENTS=gpurun_out/${TAG}kt.err python3 scripts/kernel_gaps.py gpurun_out/${TAG}kt \
      >> gpurun_out/${TAG}kt_gaps.txt
    head -3 gpurun_out/${TAG}kt_gaps.txt
  fi
fi
if [ -n "${AB:-}" ]; then
  eval "set -- $AB"
  timeout -k 10 ${T_AB:-700} bash scripts/ab_trace.sh "$1" "$2" "$3" > gpurun_out/${TAG}ab.txt 2>&1
  rc=$?; echo "ab rc=$rc"; tail -8 gpurun_out/${TAG}ab.txt; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "${CMD:-}" ]; then
  timeout -k 10 ${T_CMD:-300} bash -c "$CMD" > gpurun_out/${TAG}cmd.log 2>&1
  rc=$?; echo "cmd rc=$rc"; tail -20 gpurun_out/${TAG}cmd.log; [ $rc -eq 0 ] || exit $rc
fi
exit 0
