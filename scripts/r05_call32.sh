#!/bin/bash
# config 2 single MSM: buckets vs the (now padded) comb, ABBA x2; comb window groups
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
run() {
  env "$@" timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --extras msm > gpurun_out/b32.json 2> gpurun_out/b32.err \
    || { tail -5 gpurun_out/b32.err; exit 1; }
  python3 -c 'import json,sys;d=json.load(open("gpurun_out/b32.json"))["config2_msm"];print(sys.argv[1:], d["ms_per_step"], d.get("ms_per_step_median"), {k:v["ms_per_step"] for k,v in d["kernels"].items()})' "$@"
}
for i in 1 2; do run SPG_BIG_COMB=0; run SPG_BIG_COMB=1; run SPG_BIG_COMB=1; run SPG_BIG_COMB=0; done
run SPG_BIG_COMB=1 SPG_BIG_COMB_G=2
run SPG_BIG_COMB=1 SPG_BIG_COMB_G=1
