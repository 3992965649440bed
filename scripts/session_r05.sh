#!/bin/bash
# round-5 GPU session pieces (each step under its own time limit, chained by the caller with &&):
#   tests K            pytest -m gpu -k K
#   ab VAR "v1 v2" n   traced A/B of one switch (scripts/ab_trace.sh)
#   bench TAG ENV...   one bench line (default workload, or BENCH_ARGS) under the given env assignments
#   hipt TAG           kernel + HIP runtime API + memory-copy trace of the same proves (csv), lap events in TAG.err
#   gaps TAG           kernel trace + host lap events of 6 proves -> per-prove idle gaps by transition and by host lap
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
case "$1" in
  tests)
    timeout -k 10 ${T:-800} python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$2" \
      > gpurun_out/${TAG:-}gpu_tests.log 2>&1
    rc=$?; tail -3 gpurun_out/${TAG:-}gpu_tests.log; exit $rc ;;
  ab)
    timeout -k 10 ${T:-700} bash scripts/ab_trace.sh "$2" "$3" "$4" ;;
  bench)
    tag=$2; shift 2
    env "$@" timeout -k 10 ${T:-600} python3 bench.py ${BENCH_ARGS:---steps 20 --warmup 3} > gpurun_out/bench_$tag.json \
      2> gpurun_out/bench_$tag.err || { tail -5 gpurun_out/bench_$tag.err; exit 1; }
    tail -c 600 gpurun_out/bench_$tag.json ;;
  hipt)
    export TMPDIR=/tmp
    (cd /tmp && SPG_TRACE=2 SPG_TRACE_EVENTS=1 TRACE_REPS=4 timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace \
      --memory-copy-trace --output-format csv -d "$R/gpurun_out/kt_$2" -o kt -- python3 "$R/scripts/trace_snark.py" \
      > /dev/null 2> "$R/gpurun_out/kt_$2.err") || exit 1
    ls gpurun_out/kt_$2 ;;
  gapsb)  # kernel trace + lap events of bench.py $BENCH_ARGS (no profile pass lines needed: --steps 3)
    export TMPDIR=/tmp
    (cd /tmp && SPG_TRACE=2 SPG_TRACE_EVENTS=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv \
      -d "$R/gpurun_out/kt_$2" -o kt -- python3 "$R/bench.py" --steps 4 --warmup 1 --no-cpu-baseline --extras none \
      $BENCH_ARGS > /dev/null 2> "$R/gpurun_out/kt_$2.err") || exit 1
    ls gpurun_out/kt_$2 ;;
  gaps)
    export TMPDIR=/tmp
    (cd /tmp && SPG_TRACE=2 SPG_TRACE_EVENTS=1 TRACE_REPS=6 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv \
      -d "$R/gpurun_out/kt_$2" -o kt -- python3 "$R/scripts/trace_snark.py" > /dev/null 2> "$R/gpurun_out/kt_$2.err") || exit 1
    MARK="k_comb_accum<12, 1>" SKIP=1 python3 scripts/kernel_gaps.py gpurun_out/kt_$2 XX > gpurun_out/kt_$2_gaps.txt
    MARK="k_comb_accum<12, 1>" SKIP=1 EVENTS=gpurun_out/kt_$2.err python3 scripts/kernel_gaps.py gpurun_out/kt_$2 \
      >> gpurun_out/kt_$2_gaps.txt
    head -3 gpurun_out/kt_$2_gaps.txt ;;
esac
