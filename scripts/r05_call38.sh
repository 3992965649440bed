#!/bin/bash
# host encodings on the box: the micro, and config 4's commit timings with / without halved encodings
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
./scripts/micro/enc_batch > gpurun_out/enc_batch.txt 2>&1; cat gpurun_out/enc_batch.txt
for v in 0 1; do
  SPG_HALVED_ENC=$v SPG_TRACE=3 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --extras r1cs > gpurun_out/b38.json 2> gpurun_out/b38_$v.err || exit 1
  echo "HALVED=$v"; grep "commit rows" gpurun_out/b38_$v.err | sort | uniq -c | sort -rn | head -6
done
