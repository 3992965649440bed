#!/bin/bash
# comb tables padded to one 128-byte line per entry: parity, then A/B of the headline and configs 2 (rows) / 5
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_msm.py \
  tests/test_gpu_snark.py -k "golden or comb or bullet or round_forms" > gpurun_out/t24.log 2>&1
rc=$?; tail -3 gpurun_out/t24.log; [ $rc = 0 ] || exit $rc
for pad in 0 1 1 0; do
  SPG_COMB_PAD=$pad timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --extras rows,spark \
    > gpurun_out/b24_$pad.json 2> gpurun_out/b24_$pad.err || { tail -5 gpurun_out/b24_$pad.err; exit 1; }
  python3 -c 'import json,sys;d=json.load(open(sys.argv[1]));r=d["config2_rows"];s=d["config5_spark"];print("PAD",sys.argv[2],"snark",d["ms_per_step"],"rows",r["ms_per_step"],r["roofline"]["avg_launch_us"],r["roofline"]["traffic"],"spark",s["ms_per_step"],s["kernels"]["msm_comb"]["ms_per_step"])' gpurun_out/b24_$pad.json $pad
done
bash scripts/ab_env2.sh SPG_COMB_PAD 0 1 2 > gpurun_out/ab24_pad.txt
cat gpurun_out/ab24_pad.txt
