#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
SPG_TRACE=3 timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --extras r1cs > gpurun_out/b40.json 2> gpurun_out/b40.err || exit 1
grep "halved encodings\|commit rows=128" gpurun_out/b40.err | tail -12
