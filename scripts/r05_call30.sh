#!/bin/bash
# 8-lane batched encodings: parity, traced flush, ABBA (4 blocks)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_product_host.py tests/test_gpu_msm.py \
  tests/test_gpu_spark.py tests/test_gpu_snark.py -k "golden or commit or row_enc or oracle or comb or double" > gpurun_out/t30.log 2>&1
rc=$?; tail -3 gpurun_out/t30.log; [ $rc = 0 ] || exit $rc
SPG_TRACE=2 timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-cpu-baseline --extras rows > gpurun_out/b30t.json \
  2> gpurun_out/b30t.err || { tail -20 gpurun_out/b30t.err; exit 1; }
grep "commit queue flush\|SNARK::prove host" gpurun_out/b30t.err | tail -2
python3 -c 'import json;d=json.load(open("gpurun_out/b30t.json"));print("rows",d["config2_rows"]["ms_per_step"])'
bash scripts/ab_env2.sh SPG_HALVED_ENC 0 1 4 > gpurun_out/ab30.txt
cat gpurun_out/ab30.txt
