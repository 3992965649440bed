#!/bin/bash
# row-batch comb: window groups per scalar for the large batches (SPG_COMB_GMIN 1 / 2 / 4)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
run() {
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --extras rows > gpurun_out/b34.json 2> gpurun_out/b34.err \
    || { tail -5 gpurun_out/b34.err; exit 1; }
  python3 -c 'import json,sys;D=json.load(open("gpurun_out/b34.json"));d=D["config2_rows"];print(sys.argv[1:], "snark", D["ms_per_step"], D["device_busy_ms_per_step"], "rows", d["ms_per_step"], {k:v["ms_per_step"] for k,v in d["kernels"].items()})' "$@"
}
for i in 1 2; do run SPG_COMB_GMIN=1; run SPG_COMB_GMIN=2; run SPG_COMB_GMIN=4; done
