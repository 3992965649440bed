#!/bin/bash
# 13-bit comb windows for the 1024-generator tables too (SPG_COMB_C): headline ABBA, and the row batch
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
bash scripts/ab_env2.sh SPG_COMB_C 12 13 3 > gpurun_out/ab47.txt && cat gpurun_out/ab47.txt
for v in 12 13; do
  SPG_COMB_C=$v timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --extras rows > gpurun_out/b47.json 2> gpurun_out/b47.err || exit 1
  python3 -c 'import json,sys;d=json.load(open("gpurun_out/b47.json"))["config2_rows"];print("C",sys.argv[1],"rows",d["ms_per_step"],{k:v["ms_per_step"] for k,v in d["kernels"].items()})' $v
done
