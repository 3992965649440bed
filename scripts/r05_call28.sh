#!/bin/bash
# halved comb rows + host batched encodings: parity, rows bench, ABBA
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_msm.py tests/test_gpu_spark.py \
  tests/test_gpu_snark.py tests/test_gpu_large.py -k "golden or commit or row_enc or oracle or checked or 2e20 or comb" \
  > gpurun_out/t28.log 2>&1
rc=$?; tail -3 gpurun_out/t28.log; [ $rc = 0 ] || exit $rc
for v in 0 1; do
  SPG_HALVED_ENC=$v timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --extras rows,msm \
    > gpurun_out/b28_$v.json 2> gpurun_out/b28_$v.err || { tail -5 gpurun_out/b28_$v.err; exit 1; }
  python3 -c 'import json,sys;d=json.load(open(sys.argv[1]));r=d["config2_rows"];print("HALVED",sys.argv[2],"snark",d["ms_per_step"],"rows",r["ms_per_step"],r["kernels"])' gpurun_out/b28_$v.json $v
done
SPG_TRACE=2 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --extras none > gpurun_out/b28t.json 2> gpurun_out/b28t.err && grep "commit queue flush" gpurun_out/b28t.err | tail -2 && bash scripts/ab_env2.sh SPG_HALVED_ENC 0 1 3 > gpurun_out/ab28.txt
cat gpurun_out/ab28.txt
