#!/bin/bash
# config 4 (R1CSProof 2^22): which round-5 switch moved its wall time
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
uptime
run() {
  env "$@" timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --extras r1cs > gpurun_out/b36.json 2> gpurun_out/b36.err \
    || { tail -5 gpurun_out/b36.err; exit 1; }
  python3 -c 'import json,sys;d=json.load(open("gpurun_out/b36.json"))["config4_r1cs"];print(sys.argv[1:], d["ms_per_step"], d.get("ms_per_step_median"), d.get("device_busy_ms_per_step"))' "$@"
}
for i in 1 2; do
  run X=1; run SPG_HOST_COMMIT_MAX=0; run SPG_HALVED_ENC=0; run SPG_BCOMB_R=4; run SPG_COMB_PAD=0; run SPG_LAYER_TRIPLE=0
done
