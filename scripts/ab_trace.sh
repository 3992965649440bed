#!/bin/bash
# A/B of one environment switch with SPG_TRACE=1 host breakdowns, alternating on one box:
#   ab_trace.sh VAR "v1 v2" reps  -> per run: mean/median ms per prove, device busy, and the mean of each SNARK::prove
#   host-breakdown phase (the [spg] lines) over the run's proves (scripts/trace_avg.py)
VAR=$1; VALS=$2; REPS=${3:-3}
mkdir -p gpurun_out/abt
for r in $(seq $REPS); do
  for v in $VALS; do
    env $VAR=$v SPG_TRACE=1 timeout -k 5 150 python bench.py --steps ${AB_STEPS:-10} --warmup 3 --no-cpu-baseline \
      --extras none ${BENCH_ARGS:-} > gpurun_out/abt/b_${v}_$r.json 2> gpurun_out/abt/t_${v}_$r.txt || exit $?
    echo "$VAR=$v $(python -c 'import json,sys;d=json.load(open(sys.argv[1]));print(d["ms_per_step"], d.get("ms_per_step_median"), "dev", d.get("device_busy_ms_per_step"))' gpurun_out/abt/b_${v}_$r.json)"
    python3 scripts/trace_avg.py gpurun_out/abt/t_${v}_$r.txt input_commit block_sat block_eval pairwise perm_root total
    python3 - gpurun_out/abt/t_${v}_$r.txt <<'PY'
import re, sys
ls = [float(m.group(1)) for m in re.finditer(r"SparseMatPolyEvalProof::prove host breakdown.*?layer_sumchecks=([\d.]+)", open(sys.argv[1]).read())]
ls = ls[3:]  # the warm-up prove's three
print("  layer_sumchecks per prove (3 SPARK proofs):", round(sum(ls) / max(1, len(ls) / 3)), "us")
PY
  done
done
