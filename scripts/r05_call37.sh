#!/bin/bash
# config 4: ABBA of SPG_HOST_COMMIT_MAX 0 / 256 and of SPG_HALVED_ENC 0 / 1
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
uptime
run() {
  env "$@" timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --extras r1cs > gpurun_out/b37.json 2> gpurun_out/b37.err \
    || { tail -5 gpurun_out/b37.err; exit 1; }
  python3 -c 'import json,sys;d=json.load(open("gpurun_out/b37.json"))["config4_r1cs"];print(sys.argv[1:], d["ms_per_step"], d.get("ms_per_step_median"), d.get("device_busy_ms_per_step"))' "$@"
}
for i in 1 2 3; do run SPG_HOST_COMMIT_MAX=0; run SPG_HOST_COMMIT_MAX=256; run SPG_HOST_COMMIT_MAX=256; run SPG_HOST_COMMIT_MAX=0; done
for i in 1 2 3; do run SPG_HALVED_ENC=0; run SPG_HALVED_ENC=1; run SPG_HALVED_ENC=1; run SPG_HALVED_ENC=0; done
SPG_TRACE=3 timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --extras r1cs > gpurun_out/b37t.json 2> gpurun_out/b37t.err
grep "commit rows" gpurun_out/b37t.err | sort | uniq -c | sort -rn | head -12
